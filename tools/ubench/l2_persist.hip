// Does an XCD's L2 keep lines across a kernel boundary?  Kernel `touch` reads a region per
// XCD; kernel `reread` then reads either the same XCD's region (affine) or the next XCD's
// (shifted).  Compare the reread's duration (and FETCH_SIZE under rocprofv3 --pmc).
// Build: hipcc --offload-arch=gfx950 -O3 l2_persist.hip -o l2_persist
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ unsigned xcc_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
    return v & 7u;
}

// each workgroup reads the region of (its XCD + shift) % 8: REGION ints, strided by the
// workgroups that share its XCD (blockIdx / 8 as the rank within the group of blockIdx % 8)
__global__ void k_read(const int* a, long long region, int shift, unsigned long long* sink, unsigned* xmap) {
    const unsigned x = (xcc_id() + shift) & 7u;
    if (threadIdx.x == 0) xmap[blockIdx.x] = xcc_id();
    const int rank = blockIdx.x / 8, per = gridDim.x / 8;
    const int* r = a + (long long)x * region;
    unsigned long long s = 0;
    for (long long i = (long long)rank * blockDim.x + threadIdx.x; i < region; i += (long long)per * blockDim.x)
        s += (unsigned)r[i];
    if (s == 0xFFFFFFFFFFFFull) sink[0] = s;
}

int main() {
    const long long region = (2ll << 20) / 4;  // 2 MB per XCD
    int* a;
    unsigned long long* sink;
    unsigned* xmap;
    hipMalloc(&a, region * 8 * 4);
    hipMemset(a, 1, region * 8 * 4);
    hipMalloc(&sink, 8);
    hipMalloc(&xmap, 4096 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int grid = 1024;
    for (int rep = 0; rep < 3; ++rep) {
        for (int shift = 0; shift < 2; ++shift) {
            float best = 1e9;
            for (int it = 0; it < 20; ++it) {
                hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, a, region, 0, sink, xmap);  // touch (own XCD)
                hipEventRecord(e0);
                hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, a, region, shift, sink, xmap);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                best = ms < best ? ms : best;
            }
            printf("reread %s: best %.2f us\n", shift ? "shifted XCD" : "same XCD   ", best * 1e3);
        }
    }
    std::vector<unsigned> xm(grid);
    hipMemcpy(xm.data(), xmap, grid * 4, hipMemcpyDeviceToHost);
    int agree = 0;
    for (int b = 0; b < grid; ++b) agree += xm[b] == xm[b % 8];
    printf("blocks on the same XCD as block b%%8: %d / %d; block 0..7 on XCDs %u %u %u %u %u %u %u %u\n", agree, grid,
           xm[0], xm[1], xm[2], xm[3], xm[4], xm[5], xm[6], xm[7]);
    return 0;
}
