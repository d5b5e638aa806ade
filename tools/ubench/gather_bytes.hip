// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the engine's access patterns
// (VERDICT r4 next #5): what do the counters report per random 1-B / 4-B gather, per random
// 4-B store and per random 32-bit atomic, against a wide streaming read / write whose bytes
// are known?  MI355X_MICROARCH.md calibrates only the 16-B/lane streaming read (FETCH_SIZE
// = 1/2 of the bytes) and streaming stores (exact).
//
// Every kernel is launched REPS times with a name of its own, so a --pmc run's per-dispatch
// rows can be joined with the line this program prints for the kernel (tools/ubench_pmc.py):
//   kernel  launches  ops_per_launch  bytes_per_op  avg_us
// Gathers: lane i of the grid reads a[h(i) & (N-1)], h a 64-bit mix, N elements spanning
// 1-4 GB (far past the 256 MB Infinity Cache), so almost every op touches a line of its own;
// the "resident" case gathers from a 32 MB table (stays on die) to show whether on-die hits
// are counted.  Every loaded value feeds a sum that is stored only if impossible, so nothing
// is optimised away.
// Build: hipcc --offload-arch=gfx950 -O3 gather_bytes.hip -o gather_bytes
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned long long ull;

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

__device__ __forceinline__ ull mix(ull x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// ---- streaming (16 B per lane) ----
__global__ void k_stream_read16(const uint4* a, long long n4, unsigned* sink) {
    unsigned s = 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        s += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (s == 0x12345678u) sink[0] = s;
}
__global__ void k_stream_write16(uint4* a, long long n4) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x)
        a[i] = make_uint4((unsigned)i, 1u, 2u, 3u);
}
// ---- streaming (4 B per lane): the engine's list / row reads ----
__global__ void k_stream_read4(const unsigned* a, long long n, unsigned* sink) {
    unsigned s = 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        s += a[i];
    if (s == 0x12345678u) sink[0] = s;
}

// ---- random gathers ----
template <typename T>
__device__ __forceinline__ void gather_body(const T* a, ull mask, long long ops, unsigned salt, unsigned* sink) {
    unsigned s = 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < ops; i += (long long)gridDim.x * blockDim.x)
        s += (unsigned)a[mix((ull)i * 0x100000001ull + salt) & mask];
    if (s == 0x12345678u) sink[0] = s;
}
__global__ void k_gather4_big(const unsigned* a, ull mask, long long ops, unsigned salt, unsigned* sink) {
    gather_body(a, mask, ops, salt, sink);
}
__global__ void k_gather1_big(const unsigned char* a, ull mask, long long ops, unsigned salt, unsigned* sink) {
    gather_body(a, mask, ops, salt, sink);
}
__global__ void k_gather4_resident(const unsigned* a, ull mask, long long ops, unsigned salt, unsigned* sink) {
    gather_body(a, mask, ops, salt, sink);
}
// 8 consecutive 4-B words per op (32 B, one half of a 64-B line): a row segment
__global__ void k_gather32B_big(const uint4* a, ull mask, long long ops, unsigned salt, unsigned* sink) {
    unsigned s = 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < ops; i += (long long)gridDim.x * blockDim.x) {
        const ull j = (mix((ull)i * 0x100000001ull + salt) & mask) & ~1ull;
        const uint4 v = a[j], w = a[j + 1];
        s += v.x ^ v.y ^ v.z ^ v.w ^ w.x ^ w.y ^ w.z ^ w.w;
    }
    if (s == 0x12345678u) sink[0] = s;
}

// ---- random stores / atomics ----
__global__ void k_scatter4_big(unsigned* a, ull mask, long long ops, unsigned salt) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < ops; i += (long long)gridDim.x * blockDim.x)
        a[mix((ull)i * 0x100000001ull + salt) & mask] = (unsigned)i;
}
__global__ void k_scatter1_big(unsigned char* a, ull mask, long long ops, unsigned salt) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < ops; i += (long long)gridDim.x * blockDim.x)
        a[mix((ull)i * 0x100000001ull + salt) & mask] = (unsigned char)i;
}
__global__ void k_atomic_or4_big(unsigned* a, ull mask, long long ops, unsigned salt) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < ops; i += (long long)gridDim.x * blockDim.x)
        atomicOr(&a[mix((ull)i * 0x100000001ull + salt) & mask], 1u << (i & 31));
}

struct Timer {
    hipEvent_t a, b;
    Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
};

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = cus * 8, block = 256;
    const size_t big4 = (size_t)1 << 30;        // 2^30 u32 = 4 GB
    const size_t big1 = (size_t)1 << 30;        // 2^30 u8  = 1 GB
    const size_t res4 = (size_t)8 << 20;        // 2^23 u32 = 32 MB (stays on die)
    const size_t streamB = (size_t)2 << 30;     // 2 GB streamed
    const long long ops = 1ll << 26;            // 67M random ops per launch
    unsigned *a4, *r4, *sink;
    unsigned char* a1;
    uint4* st;
    CK(hipMalloc(&a4, big4 * 4));
    CK(hipMalloc(&a1, big1));
    CK(hipMalloc(&r4, res4 * 4));
    CK(hipMalloc(&st, streamB));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a4, 1, big4 * 4));
    CK(hipMemset(a1, 1, big1));
    CK(hipMemset(r4, 1, res4 * 4));
    CK(hipMemset(st, 1, streamB));
    CK(hipDeviceSynchronize());
    Timer t;
    printf("# kernel launches ops_per_launch bytes_per_op avg_us (grid %d x %d)\n", grid, block);
#define RUN(name, nops, bpo, launch)                                                         \
    do {                                                                                     \
        launch; /* warm */                                                                   \
        CK(hipDeviceSynchronize());                                                          \
        CK(hipEventRecord(t.a));                                                             \
        for (int r_ = 0; r_ < reps; ++r_) launch;                                            \
        CK(hipEventRecord(t.b));                                                             \
        CK(hipEventSynchronize(t.b));                                                        \
        float ms_ = 0;                                                                       \
        CK(hipEventElapsedTime(&ms_, t.a, t.b));                                             \
        printf("%s %d %lld %d %.3f\n", name, reps + 1, (long long)(nops), (int)(bpo), ms_ * 1e3 / reps); \
        fflush(stdout);                                                                      \
    } while (0)
    const long long n4 = (long long)(streamB / 16);
    RUN("k_stream_read16", streamB / 16, 16, hipLaunchKernelGGL(k_stream_read16, dim3(grid), dim3(block), 0, 0, st, n4, sink));
    RUN("k_stream_write16", streamB / 16, 16, hipLaunchKernelGGL(k_stream_write16, dim3(grid), dim3(block), 0, 0, st, n4));
    RUN("k_stream_read4", streamB / 4, 4,
        hipLaunchKernelGGL(k_stream_read4, dim3(grid), dim3(block), 0, 0, (const unsigned*)st, (long long)(streamB / 4), sink));
    unsigned salt = 1;
    RUN("k_gather4_big", ops, 4,
        hipLaunchKernelGGL(k_gather4_big, dim3(grid), dim3(block), 0, 0, a4, (ull)(big4 - 1), ops, salt++, sink));
    RUN("k_gather1_big", ops, 1,
        hipLaunchKernelGGL(k_gather1_big, dim3(grid), dim3(block), 0, 0, a1, (ull)(big1 - 1), ops, salt++, sink));
    RUN("k_gather4_resident", ops, 4,
        hipLaunchKernelGGL(k_gather4_resident, dim3(grid), dim3(block), 0, 0, r4, (ull)(res4 - 1), ops, salt++, sink));
    RUN("k_gather32B_big", ops, 32,
        hipLaunchKernelGGL(k_gather32B_big, dim3(grid), dim3(block), 0, 0, (const uint4*)a4, (ull)(big4 / 4 - 1), ops, salt++, sink));
    RUN("k_scatter4_big", ops, 4,
        hipLaunchKernelGGL(k_scatter4_big, dim3(grid), dim3(block), 0, 0, a4, (ull)(big4 - 1), ops, salt++));
    RUN("k_scatter1_big", ops, 1,
        hipLaunchKernelGGL(k_scatter1_big, dim3(grid), dim3(block), 0, 0, a1, (ull)(big1 - 1), ops, salt++));
    RUN("k_atomic_or4_big", ops, 4,
        hipLaunchKernelGGL(k_atomic_or4_big, dim3(grid), dim3(block), 0, 0, a4, (ull)(big4 - 1), ops, salt++));
    CK(hipDeviceSynchronize());
    return 0;
}
