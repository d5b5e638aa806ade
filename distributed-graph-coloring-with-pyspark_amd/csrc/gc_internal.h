// gc_internal.h -- shared definitions for the gfx950 colouring engine (not part of the ABI).
//
// Layout in HBM (per gc_graph, all resident for the handle's lifetime):
//   rp    int64[n+1]   CSR row offsets (file positions, lists as listed)
//   col   int32[nnz]   neighbour positions
//   deg   int32[n]     rp[v+1]-rp[v] (hot: rank compares, binning)
//   trp/tcol           in-neighbour CSR for the frontier push (aliases rp/col when symmetric)
// Run state (reused across gc_color calls):
//   color int32[n], cround int32[n], key u64[n] = (cand<<32 | deg), jp u8[n] (JP state),
//   inF   u32[n/32]    bit = coloured or already in the frontier (claim bitmap)
//   lists int32[n]     frontier (cur/next), heavy, wide, undecided x2, seed lists
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned long long ull;

#define GC_WAVE 64
#define GC_BLOCK 256
#define GC_WAVES_PER_BLOCK (GC_BLOCK / GC_WAVE)
// Vertices with deg > GC_HEAVY_T take the workgroup-per-vertex path.
#define GC_HEAVY_T 2048
// per-wave LDS staging capacity for list appends
#define GC_STAGE_CAP 512

#define GC_KEY_INVALID 0xFFFFFFFF00000000ull
#define GC_JP_UND 0
#define GC_JP_IN 1
#define GC_JP_OUT 2

// Device-resident counters.  Zeroed / read by the host engine around each launch group.
struct DevCtl {
    ull fcnt[2];       // frontier sizes (ping-pong: current / next)
    ull heavy_cnt;     // heavy proposers (this round)
    ull wide_cnt;      // light proposers whose mex >= 64
    ull und_cnt[2];    // undecided lists (ping-pong)
    ull seed_cnt[2];   // seed lists: [0] light, [1] heavy
    ull accepted;      // committed this round
    ull failcnt;       // proposers with mex >= k
    long long maxmex;  // max candidate this round (-1)
    long long maxcolor;// max colour committed so far
    ull seedkey;       // argmax (deg << 32 | pos) over uncoloured
    ull uncolored;     // init: #uncoloured; validate: #uncoloured
    ull conflicts;     // validate
    ull list_cnt;      // E1: compacted uncoloured list
    ull nseeds;        // E1 seeds planted
    ull sumdeg[8];     // per kernel class: sum of degrees touched (algorithmic bytes)
    ull nvert[8];      // per kernel class: vertices processed
};

__device__ __forceinline__ int gc_lane() { return (int)__lane_id(); }
__device__ __forceinline__ ull gc_lanemask_lt() { return (1ull << gc_lane()) - 1ull; }

__device__ __forceinline__ void gc_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int gc_wave_incl_scan(int x) {
    const int l = gc_lane();
#pragma unroll
    for (int o = 1; o < GC_WAVE; o <<= 1) {
        int y = __shfl_up(x, o, GC_WAVE);
        if (l >= o) x += y;
    }
    return x;
}

template <typename T>
__device__ __forceinline__ T gc_wave_max(T x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        T y = __shfl_xor(x, o, GC_WAVE);
        x = y > x ? y : x;
    }
    return x;
}

template <typename T>
__device__ __forceinline__ T gc_wave_sum(T x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, GC_WAVE);
    return x;
}

// Owner lane of edge slot e inside a wave chunk: max j with excl_j <= e (excl sorted).
// Must be called with all 64 lanes active.
__device__ __forceinline__ int gc_owner(int excl, int e) {
    int o = 0;
#pragma unroll
    for (int step = 32; step > 0; step >>= 1) {
        int x = __shfl(excl, o + step, GC_WAVE);
        if (x <= e) o += step;
    }
    return o;
}

// Per-wave append staging in LDS: one global atomic per GC_STAGE_CAP entries instead of
// one per wave-instruction (a single counter saturates at ~88 returning atomics/us).
struct GcStage {
    int* buf;
    int cnt;  // wave-uniform
};

__device__ __forceinline__ void gc_stage_flush(GcStage& s, int* out, ull* out_cnt) {
    gc_wave_sync();
    if (s.cnt == 0) return;
    ull base = 0;
    if (gc_lane() == 0) base = atomicAdd(out_cnt, (ull)s.cnt);
    base = __shfl(base, 0, GC_WAVE);
    for (int i = gc_lane(); i < s.cnt; i += GC_WAVE) out[base + i] = s.buf[i];
    gc_wave_sync();
    s.cnt = 0;
}

// All 64 lanes must call; pred per lane.
__device__ __forceinline__ void gc_stage_push(GcStage& s, bool pred, int val, int* out, ull* out_cnt) {
    const ull m = __ballot(pred);
    const int n = __popcll(m);
    if (n == 0) return;
    if (s.cnt + n > GC_STAGE_CAP) gc_stage_flush(s, out, out_cnt);
    if (pred) s.buf[s.cnt + __popcll(m & gc_lanemask_lt())] = val;
    s.cnt += n;
}

// Wave-aggregated direct append (rare lists).  All lanes must call.
__device__ __forceinline__ void gc_wave_append(bool pred, int val, int* out, ull* out_cnt) {
    const ull m = __ballot(pred);
    if (m == 0) return;
    ull base = 0;
    const int leader = __ffsll((long long)m) - 1;
    if (gc_lane() == leader) base = atomicAdd(out_cnt, (ull)__popcll(m));
    base = __shfl(base, leader, GC_WAVE);
    if (pred) out[base + __popcll(m & gc_lanemask_lt())] = val;
}

// Block reductions into global counters (one atomic per block).
__device__ __forceinline__ void gc_block_add(ull* dst, ull v, ull* lds_scratch) {
    v = gc_wave_sum(v);
    const int w = threadIdx.x / GC_WAVE;
    if (gc_lane() == 0) lds_scratch[w] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        ull t = 0;
        for (int i = 0; i < (int)(blockDim.x / GC_WAVE); ++i) t += lds_scratch[i];
        if (t) atomicAdd(dst, t);
    }
    __syncthreads();
}

__device__ __forceinline__ void gc_block_max(long long* dst, long long v, long long* lds_scratch) {
    v = gc_wave_max(v);
    const int w = threadIdx.x / GC_WAVE;
    if (gc_lane() == 0) lds_scratch[w] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        long long t = lds_scratch[0];
        for (int i = 1; i < (int)(blockDim.x / GC_WAVE); ++i) t = lds_scratch[i] > t ? lds_scratch[i] : t;
        atomicMax(dst, t);
    }
    __syncthreads();
}

__device__ __forceinline__ uint32_t gc_key_cand(ull k) { return (uint32_t)(k >> 32); }
__device__ __forceinline__ uint32_t gc_key_deg(ull k) { return (uint32_t)k; }
__device__ __forceinline__ ull gc_make_key(uint32_t cand, uint32_t deg) { return ((ull)cand << 32) | deg; }

// rank order of coloring.py:64 (stable sort by deg of a file-ordered group): (deg, pos) asc
__device__ __forceinline__ bool gc_rank_lt(uint32_t du, int u, uint32_t dv, int v) {
    return du < dv || (du == dv && u < v);
}
