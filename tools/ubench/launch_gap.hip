// What does one dependent kernel boundary cost on one stream?  A colouring round on R-MAT is
// ~7 launches (propose, propose_block, resolve, sweep, commit, commit_big, close) and the
// round-2 trace shows ~5.5 us median gaps at some boundaries and none at others
// (profiles/latest/rmat24/gaps.txt).  Each pattern below enqueues REPS launches back to back
// and reports the wall time per launch (hipEvents around the chain), so the per-boundary
// cost can be read per shape:
//   tiny        1 workgroup of 64 lanes, 8-byte argument
//   tiny_args   the same with a 768-byte argument struct (the engine's GDev + GLists are ~700 B)
//   grid_noop   2048 x 256 that return at once (reading a device flag, as a halted round does)
//   grid_args   the same with the 768-byte struct
//   grid_write  2048 x 256, one agent-scope store per workgroup
//   grid_lds    2048 x 256 with 48 KB of static LDS (occupancy-limited launch)
//   alt         grid_write and tiny alternating (a close after a commit)
//   graph_alt   alt captured once in a hipGraph and replayed
// Build: hipcc --offload-arch=gfx950 -O3 launch_gap.hip -o launch_gap ; run: ./launch_gap [REPS]
// (alt and graph_alt print the cost of one PAIR of launches)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

struct Big {
    long long w[96];  // 768 bytes
};

__global__ void k_tiny(int* flag) {
    if (threadIdx.x == 0 && *flag == 12345) flag[1] = 1;
}
__global__ void k_tiny_args(Big b, int* flag) {
    if (threadIdx.x == 0 && *flag == (int)b.w[95]) flag[1] = 1;
}
__global__ void k_grid_noop(int* flag) {
    if (*flag != 12345) return;
    flag[2] = 1;
}
__global__ void k_grid_args(Big b, int* flag) {
    if (*flag != (int)b.w[7]) return;
    flag[2] = 1;
}
__global__ void k_grid_write(unsigned* out) {
    if (threadIdx.x == 0) __hip_atomic_store(out + blockIdx.x, blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void k_grid_lds(unsigned* out) {
    __shared__ unsigned s[12 * 1024];  // 48 KB
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = s[(blockIdx.x + 1) & 255];
}

template <typename F>
float per_launch_us(F enqueue, int reps, hipStream_t s) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    enqueue(16);  // warm-up
    CK(hipStreamSynchronize(s));
    float best = 1e30f;
    for (int t = 0; t < 5; ++t) {
        CK(hipEventRecord(e0, s));
        enqueue(reps);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return best * 1000.f / (float)reps;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 2000;
    const int grid = 2048;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int* flag;
    unsigned* out;
    CK(hipMalloc(&flag, 64));
    CK(hipMemset(flag, 0, 64));
    CK(hipMalloc(&out, sizeof(unsigned) * grid));
    Big b{};
    for (int i = 0; i < 96; ++i) b.w[i] = i + 1;
    printf("pattern      us/launch  (REPS=%d, best of 5)\n", reps);
    printf("tiny         %8.2f\n", per_launch_us([&](int n) {
        for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, flag);
    }, reps, s));
    printf("tiny_args    %8.2f\n", per_launch_us([&](int n) {
        for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_tiny_args, dim3(1), dim3(64), 0, s, b, flag);
    }, reps, s));
    printf("grid_noop    %8.2f\n", per_launch_us([&](int n) {
        for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_grid_noop, dim3(grid), dim3(256), 0, s, flag);
    }, reps, s));
    printf("grid_args    %8.2f\n", per_launch_us([&](int n) {
        for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_grid_args, dim3(grid), dim3(256), 0, s, b, flag);
    }, reps, s));
    printf("grid_write   %8.2f\n", per_launch_us([&](int n) {
        for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_grid_write, dim3(grid), dim3(256), 0, s, out);
    }, reps, s));
    printf("grid_lds     %8.2f\n", per_launch_us([&](int n) {
        for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_grid_lds, dim3(grid), dim3(256), 0, s, out);
    }, reps, s));
    printf("alt (pair)   %8.2f\n", 2.f * per_launch_us([&](int n) {
        for (int i = 0; i < n / 2; ++i) {
            hipLaunchKernelGGL(k_grid_write, dim3(grid), dim3(256), 0, s, out);
            hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, flag);
        }
    }, reps, s));
    {  // the same pair chain captured in a graph (64 pairs per graph), replayed
        const int per = 64;
        hipGraph_t gr;
        hipGraphExec_t ex;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < per; ++i) {
            hipLaunchKernelGGL(k_grid_write, dim3(grid), dim3(256), 0, s, out);
            hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, flag);
        }
        CK(hipStreamEndCapture(s, &gr));
        CK(hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0));
        const int greps = (reps / (2 * per) > 0 ? reps / (2 * per) : 1) * 2 * per;  // whole graphs
        printf("graph_alt    %8.2f\n", 2.f * per_launch_us([&](int n) {
            for (int i = 0; i < n / (2 * per); ++i) CK(hipGraphLaunch(ex, s));
        }, greps, s));
        CK(hipGraphExecDestroy(ex));
        CK(hipGraphDestroy(gr));
    }
    CK(hipStreamSynchronize(s));
    CK(hipFree(flag));
    CK(hipFree(out));
    CK(hipStreamDestroy(s));
    return 0;
}
