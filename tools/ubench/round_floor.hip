// What can a small colouring round cost at best?  (a resident
// multi-round kernel confined to one XCD for the small-round tail.)
//
// A model round is six dependent phases -- the engine's propose, first JP sweep, asynchronous
// sweeps, commit, big-row commit and close.  Phase p of round r reads the item list the
// previous phase wrote and, per item, makes G dependent random gathers into a table
// (a list entry -> row -> neighbour bytes chain), then writes the item's result for the next
// phase.  Three ways to run R rounds of W items:
//   kernels  six launches per round on a 1024-workgroup grid (the engine today);
//   xcd      ONE launch for all R rounds; only workgroups with blockIdx % 8 == 0 work (the
//            hardware dispatches workgroups to the 8 XCDs round-robin, checked with
//            HW_REG_XCC_ID), so the working set stays in one XCD's L2; phases are separated
//            by a barrier on a counter in that L2 (agent-scope atomics), cross-workgroup data
//            is read with agent-scope loads (L1 bypassed, L2-served);
//   grid     ONE launch, every XCD, phases separated by a device-wide barrier (release: each
//            wave's stores drained, L2 written back; acquire: L1 and L2 invalidated).
// Prints microseconds per round for each mode and W, and whether every active workgroup of
// the xcd mode shared one XCD.  Bounded spins: a barrier that waits more than ~50 ms gives up
// and reports (the grid is sized to be co-resident, so it never should).
// Build: hipcc --offload-arch=gfx950 -O3 round_floor.hip -o round_floor
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

constexpr int PHASES = 6;
constexpr int G = 4;  // dependent gathers per item and phase

__device__ __forceinline__ unsigned xcc_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
    return v & 7u;
}
__device__ __forceinline__ int ald(const int* p) {
    return __hip_atomic_load(const_cast<int*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one phase over items [i0, W) strided by `step`; AG: cross-workgroup reads agent-scope
template <bool AG>
__device__ __forceinline__ void phase(const int* __restrict__ tab, int mask, const int* in, int* out, int W, int i0,
                                      int step) {
    for (int i = i0; i < W; i += step) {
        int v = AG ? ald(in + i) : in[i];
#pragma unroll
        for (int k = 0; k < G; ++k) v = tab[(v * 2654435761u + k) & mask];
        out[i] = v & mask;
    }
}

__global__ void k_phase(const int* tab, int mask, const int* in, int* out, int W) {
    phase<false>(tab, mask, in, out, W, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x);
}

// barrier on a monotonic counter: every wave drains its stores, lane 0 of each workgroup
// arrives, then polls until `target` arrivals; GRID adds the L2 write-back / invalidate
template <bool GRID>
__device__ __forceinline__ bool barrier(unsigned* cnt, unsigned target, int* err) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    bool ok = true;
    if (threadIdx.x == 0) {
        // xcd: the stores are in the shared L2 once drained (L1 is write-through) and the
        // readers bypass L1, so relaxed atomics suffice -- an agent-scope release / acquire
        // would write back and invalidate the L2 the mode is meant to keep
        if (GRID) __threadfence();
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        long long t0 = wall_clock64();
        while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (wall_clock64() - t0 > 5000000) {  // ~50 ms at 100 MHz
                *err = 1;
                ok = false;
                break;
            }
        }
        if (GRID) __threadfence();
    }
    __syncthreads();
    return ok;
}

__global__ void k_rounds_xcd(const int* tab, int mask, int* bufs, int W, int R, unsigned* cnt, int* err,
                             unsigned* xmap) {
    if (blockIdx.x % 8) return;  // one XCD's workgroups
    const int vb = blockIdx.x / 8, nvb = gridDim.x / 8;
    if (threadIdx.x == 0) xmap[vb] = xcc_id();
    unsigned target = 0;
    for (int r = 0; r < R; ++r)
        for (int p = 0; p < PHASES; ++p) {
            const int* in = bufs + (size_t)(p % 2) * W;
            int* out = bufs + (size_t)((p + 1) % 2) * W;
            phase<true>(tab, mask, in, out, W, vb * blockDim.x + threadIdx.x, nvb * blockDim.x);
            target += nvb;
            if (!barrier<false>(cnt, target, err)) return;
        }
}

__global__ void k_rounds_grid(const int* tab, int mask, int* bufs, int W, int R, unsigned* cnt, int* err) {
    unsigned target = 0;
    for (int r = 0; r < R; ++r)
        for (int p = 0; p < PHASES; ++p) {
            const int* in = bufs + (size_t)(p % 2) * W;
            int* out = bufs + (size_t)((p + 1) % 2) * W;
            phase<false>(tab, mask, in, out, W, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x);
            target += gridDim.x;
            if (!barrier<true>(cnt, target, err)) return;
        }
}

int main(int argc, char** argv) {
    const int R = argc > 1 ? atoi(argv[1]) : 200;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int tab_n = 1 << 24;  // 64 MB table: misses L2, mostly Infinity-Cache hits
    const int mask = tab_n - 1;
    const int Wmax = 1 << 16;
    std::vector<int> h(tab_n);
    unsigned x = 12345;
    for (int i = 0; i < tab_n; ++i) {
        x = x * 1664525u + 1013904223u;
        h[i] = (int)(x & (unsigned)mask);
    }
    int *tab, *bufs, *err;
    unsigned *cnt, *xmap;
    CK(hipMalloc(&tab, sizeof(int) * tab_n));
    CK(hipMalloc(&bufs, sizeof(int) * 2 * Wmax));
    CK(hipMalloc(&err, sizeof(int)));
    CK(hipMalloc(&cnt, sizeof(unsigned)));
    CK(hipMalloc(&xmap, sizeof(unsigned) * 4096));
    CK(hipMemcpy(tab, h.data(), sizeof(int) * tab_n, hipMemcpyHostToDevice));
    CK(hipMemcpy(bufs, h.data(), sizeof(int) * 2 * Wmax, hipMemcpyHostToDevice));
    CK(hipMemset(err, 0, sizeof(int)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int xcd_grid = 8 * cus / 8 * 2;  // 2 workgroups per CU of one XCD (cus / 8 CUs per XCD)
    const int grid_grid = cus;              // one workgroup per CU, all co-resident
    printf("# us per round (%d phases x %d dependent gathers per item), %d rounds; CUs %d\n", PHASES, G, R, cus);
    printf("# W  kernels(1024 WGs)  xcd(%d WGs on one XCD)  grid(%d WGs, device barrier)\n", xcd_grid / 8, grid_grid);
    for (int W : {64, 512, 2048, 8192, 16384, 65536}) {
        float ms_k = 0, ms_x = 0, ms_g = 0;
        for (int rep = 0; rep < 2; ++rep) {  // the second repetition is reported
            CK(hipEventRecord(e0));
            for (int r = 0; r < R; ++r)
                for (int p = 0; p < PHASES; ++p)
                    hipLaunchKernelGGL(k_phase, dim3(1024), dim3(256), 0, 0, tab, mask, bufs + (size_t)(p % 2) * W,
                                       bufs + (size_t)((p + 1) % 2) * W, W);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms_k, e0, e1));
            CK(hipMemset(cnt, 0, sizeof(unsigned)));
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_rounds_xcd, dim3(xcd_grid), dim3(256), 0, 0, tab, mask, bufs, W, R, cnt, err, xmap);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms_x, e0, e1));
            CK(hipMemset(cnt, 0, sizeof(unsigned)));
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_rounds_grid, dim3(grid_grid), dim3(256), 0, 0, tab, mask, bufs, W, R, cnt, err);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms_g, e0, e1));
        }
        int herr = 0;
        CK(hipMemcpy(&herr, err, sizeof(int), hipMemcpyDeviceToHost));
        printf("%6d %10.2f %10.2f %10.2f%s\n", W, ms_k * 1e3 / R, ms_x * 1e3 / R, ms_g * 1e3 / R,
               herr ? "  (a barrier gave up)" : "");
        fflush(stdout);
    }
    std::vector<unsigned> xm(xcd_grid / 8);
    CK(hipMemcpy(xm.data(), xmap, sizeof(unsigned) * xm.size(), hipMemcpyDeviceToHost));
    int same = 0;
    for (unsigned v : xm) same += v == xm[0];
    printf("xcd mode: %d of %zu active workgroups on XCD %u\n", same, xm.size(), xm[0]);
    return 0;
}
