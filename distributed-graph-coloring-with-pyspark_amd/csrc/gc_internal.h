// gc_internal.h -- shared definitions for the gfx950 colouring engine (not part of the ABI).
//
// Layout in HBM (per gc_graph, all resident for the handle's lifetime):
//   rp    int64[n+1]   CSR row offsets (file positions, lists as listed)
//   col   int32[nnz]   neighbour positions
//   deg   int32[n]     rp[v+1]-rp[v] (binning, algorithmic-byte accounting)
//   nlow  int32[n]     rows are stored lower-rank neighbours first (rank = (deg, pos),
//                      static); nlow[v] of them -- the only ones a JP sweep reads
//   trp/tcol           in-neighbour CSR for the frontier push (aliases rp/col when symmetric)
// Run state (reused across gc_color calls):
//   color int32[n]  cround int32[n] (written only when the caller asks for it)
//   cand  int32[n]  candidate of the current round, only for candidates >= 62
//   c8    u8[n]     colour mirror gathered by propose: colour, GC_C8_NONE (uncoloured) or
//                   GC_C8_BIG (colour >= 254, then color[] holds it); color[] itself is
//                   rebuilt from c8 once at the end (k_finalize)
//   c4    u32[n/8]  nibble mirror of c8, rebuilt for big rounds while colours < 14
//   k8    u8[n]     proposal byte gathered by resolve: cand6 << 2 | JP state
//   inF   u32[n/32] bit = coloured or already in the frontier (claim bitmap)
//   lists int32[n]  frontier (x2), heavy, wide, undecided (x3 light, x3 heavy), seeds, E1
// The narrow mirrors shrink the footprint of the per-edge random gathers against the
// 4 MB L2 per XCD (C2: 5-10 MB for propose and resolve instead of 40-80 MB).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned long long ull;

#define GC_WAVE 64
#define GC_BLOCK 256
#define GC_WAVES_PER_BLOCK (GC_BLOCK / GC_WAVE)
// Vertices with deg > GC_HEAVY_T take the workgroup-per-vertex path.
#define GC_HEAVY_T 2048
// hubs (gc_hubs.hip): default threshold, bitmap words (4096 colours)
#define GC_HUB_T 512
#define GC_HUB_W 128
#define GC_HUB_LONG 16384   // hub-start sweep: longer hlow rows are first-read by the whole grid
#define GC_HCH 1024         // entries per static chunk of an hlow row (one wave each)
#ifndef GC_HUB_UNR
#define GC_HUB_UNR 8        // hub row walk (gc_hub_jp_wave): entries per lane in flight
#endif
#define GC_HUB_NOT_STARTED (1ll << 40)
#define GC_TAIL_HMAX_HUB 128
#define GC_BIGROW 2048       // a winner with longer in-rows (+ hub pushes) is walked by the whole grid (k_commit_big); 4096 -> 2048: R-MAT-24 224 -> 217 ms
// per-wave LDS staging capacity for list appends
#define GC_STAGE_CAP 512
// fixed grid of the device-predicated round kernels (grid-stride over device counts)
#define GC_ROUND_GRID 1024
#ifndef GC_TAIL_MAX
#define GC_TAIL_MAX 1024  // JP sweeps over at most this many light vertices run in k_sweep_tail (GDev.tail_lmax)
#endif
#define GC_LOOP_MAX 65536 // ... and over at most this many light vertices in k_sweep_loop
#define GC_LOOP_HMAX 16384 //   (hubs)
#define GC_TAIL_HMAX 4    // ... and at most this many heavy ones
#ifndef GC_CHECKS
#define GC_CHECKS 0  // debug builds (tools/build_variant.sh NAME -DGC_CHECKS=1): range checks in k_commit
#endif
#ifndef GC_SWEEP_STATS
#define GC_SWEEP_STATS 0  // sumdeg / nvert counters of the JP sweeps (no §8d credit, diagnostics only):
                          // their end-of-kernel reduction cost R-MAT-24 236 -> 228 ms
#endif
#ifndef GC_TAIL_WAVES
#define GC_TAIL_WAVES 4   // waves of k_sweep_tail's one workgroup (4, 8 or 16; GDev.tail_nw)
#endif
#define GC_BLOCK_GRID 1024
#define GC_STAT_SLOTS 256
#define GC_ACC_SLOTS 256
#define GC_TICK_WORDS 72   // k_commit_big's arrival tickets after the winner slots: 8 residues x 8 words, top   // commit's winner count, summed by k_close  // per-class algorithmic-byte counters spread over slots (k_stat_reduce)
// dynamic LDS words of the workgroup-per-vertex mex bitmap (128 Ki colours per window)
#define GC_MEX_WORDS 4096

#define GC_C8_NONE 0xFFu
#define GC_C8_BIG 0xFEu
#define GC_JP_UND 0
#define GC_JP_IN 1
#define GC_JP_OUT 2

// halt codes of the device round pipeline (DevCtl.halt)
#define GC_RUN 0
#define GC_H_DONE 1
#define GC_H_FAILED 2
#define GC_H_STALLED 3
#define GC_H_RESEED 4   // zero proposers with uncoloured vertices left: host runs E1
#define GC_H_SWEEPS 5   // JP not finished after the enqueued sweeps: host adds sweeps
#define GC_H_ROUNDCAP 6 // per-round record buffer full
#define GC_H_SEAM 7     // shards: a fused propose seam was not applied (a rank halted, or its deltas overflowed)
#define GC_SEAM_HDR 5   // header words in front of a shard seam's payload (k_shard_pack)

// commit modes (bookkeeping done by the last workgroup)
#define GC_CM_ROUND 0
#define GC_CM_INIT 1
#define GC_CM_RESEED 2
#define GC_CM_SHARD 3   // sharded round: the rank's frontier, no halt / sweep checks
// k_commit nsweeps in GC_CM_SHARD mode: the replicated hub JP ran asynchronously
// (gc_shard_start_hubs_async): check that it converged first, else halt with GC_H_SWEEPS
#define GC_SHARD_CHECK (-3)

// kinds of exchanged deltas (sharded engine)
#define GC_KIND_CAND 0
#define GC_KIND_STATE 1
#define GC_KIND_COLOUR 2

// per-round record (device), copied to gc_stats at the end
struct RoundRec {
    long long U, F, maxmex, accepted, seeds, sweeps;
};

// Device-resident control block.  Counters are updated with device-scope atomics; the
// round state (cur, round, U, halt) is advanced by the last workgroup of each commit.
struct DevCtl {
    int halt;          // GC_RUN or a GC_H_* code; every round kernel returns at once if set
    int cur;           // frontier slot of the current round
    long long round;   // index of the current round (records written so far)
    long long U;       // uncoloured at the start of the current round
    long long kbound;  // k of graph_coloring(graph, k); < 0 unbounded
    int e1;            // E1 re-seed enabled
    int pad0;
    long long rcap;    // capacity of the round record buffer
    long long rbase;   // absolute round index of record slot 0 (host drains full buffers)
    long long fail_round;
    long long fail_count;
    ull fcnt[2];      // frontier sizes (ping-pong: current / next)
    ull heavy_cnt;     // heavy proposers (this round)
    ull wide_cnt;      // light proposers whose mex >= 64
    ull und_cnt[3];    // undecided light lists (rotating)
    ull undh_cnt[3];   // undecided heavy lists (rotating)
    ull seed_cnt[2];   // seed lists: [0] light, [1] heavy
    ull accepted;      // committed this round
    ull failcnt;       // proposers with mex >= k
    long long maxmex;  // max candidate this round (-1)
    long long maxcolor;// max colour committed so far
    ull seedkey;       // argmax (deg << 32 | pos) over uncoloured
    ull uncolored;     // init: #uncoloured; validate: #uncoloured
    ull conflicts;     // validate
    ull list_cnt;      // E1: compacted uncoloured list
    ull nx_failcnt;    // fused commit (k_commit<1>): next round's proposers with mex >= k
    ull dcnt;          // sharded: deltas written this phase
    ull rwin_cnt;      // sharded: other ranks' winners of this round, received as state deltas
    ull bigw_cnt;      // winners deferred to k_commit_big this commit
    long long sweeps;  // JP sweeps that found work in the current round (first included)
    long long sweep_total;  // sum over rounds of sweeps beyond the first
    long long maxdepth;     // max JP passes of a round (first sweep included)
    long long lastdepth;    // JP passes of the last closed round
    long long sweeps_enq;   // GC_H_SWEEPS: sweeps enqueued for the halted round
    long long bigsweeps;    // this round: last full-grid sweep whose input exceeded the tail limits
    long long lastbig;      // bigsweeps of the last closed round (host: full-grid sweeps to enqueue)
    long long tail_last;    // this round: index of the last sweep run (k_sweep_tail)
    long long hugesweeps;   // this round: last sweep whose input exceeded the loop kernel's limits
    long long lasthuge;     // hugesweeps of the last closed round (host: full-grid sweeps to enqueue)
    long long loop_last;    // this round: index of the last sweep run by k_sweep_loop (0: none)
    unsigned bar;           // k_sweep_loop's grid barrier: arrivals, monotonic over a colouring
    unsigned bar_base;      //   arrivals at the end of the previous k_sweep_loop launch
    int loop_err;           //   a barrier wait gave up (never expected; the host reports it)
    int pad2;
    int use_c4;             // this round's propose gathers the nibble mirror
    int resort;             // this round's frontier is rebuilt in vertex order
    int fsort_all;          // variant B: rebuild the list as EVERY claimed uncoloured vertex, and count it
    int pull_off;           // never pull the frontier (GC_NO_PULL: A/B measurements)
    int sorted;             // the current frontier list is in vertex order (built by k_front_*)
    int want_cround;        // commit records the round each vertex was coloured in
    int pad1;
    long long hub_start;    // hubs on: the sweep of this round that started the hubs' JP (the lights had converged)
    long long nx_maxmex;    // fused commit: next round's max candidate (k_close moves both into place)
    ull bcnt[9];            // variant B work lists: kind (0 light admission, 1 heavy admission, 2 eviction) x 3 rotating slots
    ull xhub_cnt;           // shards with replicated hubs: frontier hubs this rank does not own (not counted in F)
    int lights_hold;        // shards: the hub JP waits for every rank's lights (cleared by gc_shard_release_hubs)
    int pad4;
    int proposed;           // the current round's proposals were made by the last (fused) commit
    int pad3;
    long long acc_last;     // shards: winners of the last finished round (k_shard_reset keeps them for the seam header)
    long long acc_round;    // shards: round + 1 whose reset took acc_last (a repeated propose seam keeps it)
    ull async_done[2];      // k_sweep_async: light vertices decided by this launch (slot = launch parity; the
                            //   launch zeroes the other slot for the next one)
    ull async_aborts;       // k_sweep_async launches that gave up at their time budget (stats)
    int async_abort[2];     // k_sweep_async: some wave hit the budget (slot = launch parity)
    long long dbg[4];       // GC_CHECKS builds: the first out-of-range value a checked kernel met (code, a, b, c)
    ull sumdeg[8];     // per kernel class: sum of degrees touched (algorithmic bytes)
    ull nvert[8];      // per kernel class: vertices processed
    // the hub core (gc_core.hip): the uncoloured hubs' adjacency as bitsets, built once a round's
    // uncoloured hubs fit; k_hub_core then decides a round's hubs in one workgroup
    long long core_round;   // the round whose hubs k_hub_core decided (k_sweep_async returns at once); -1 none
    ull core_cnt;           // build: uncoloured hubs counted
    int core_state;         // GC_CORE_NONE / _FAILED (more uncoloured hubs than the cap) / _READY
    int core_n;             // hubs in the core (core index = rank order among them)
    long long core_handled; // rounds decided by k_hub_core (stats)
    long long core_iters_sum;  // their iterations (the chain: the most winners of one class), summed
    long long core_iters_max;  //   and the largest
};
#define GC_CORE_NONE 0
#define GC_CORE_FAILED 2
#define GC_CORE_READY 4

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

// Vertices per wave chunk for a list of cnt entries spread over `waves` waves: 64 for
// big lists (bandwidth), down to 1 for short ones (one vertex per wave, its edges over
// the lanes: a tail sweep costs one dependent gather instead of ceil(64*deg/64)).
#ifndef GC_VPW_MAX
#define GC_VPW_MAX 64
#endif
__device__ __forceinline__ int gc_vpw(long long cnt, long long waves) {
    long long per = (cnt + waves - 1) / waves;
    int v = 1;
    while (v < GC_VPW_MAX && v < per) v <<= 1;
    return v;
}

// Per-wave append staging in LDS: one global atomic per GC_STAGE_CAP entries instead of
// one per wave-instruction (a single counter saturates at ~88 returning atomics/us).
// Every list a stage flushes into holds `cap` entries (int32[n]); a flush whose base + count
// would pass it writes nothing, sets DevCtl.loop_err = GC_LERR_LIST, which the host reports
// as GC_EHIP, and halts the pipeline (DevCtl.halt = GC_H_STALLED): the list's counter is left
// past its capacity, and every later kernel returns at once instead of reading the list up to
// that count.  A wrong base becomes a reported error, never an aperture fault.
#define GC_LERR_LIST 5
#define GC_LERR_INL 6  // k_propose<1>: a hub bitmap no longer covers the colours in use
struct GcStage {
    int* buf;
    int cnt;  // wave-uniform
    long long cap;  // entries of the destination list
    int* err;       // DevCtl.loop_err
    int* halt;      // DevCtl.halt
};

// A commit that closes its own round (k_commit with tclose) counts arrivals in the high bits
// of the next frontier's counter (gc_stage_flush_ticket: + 2^40 per workgroup), so a wave
// whose stage overflows mid-launch reads back a count that carries the tickets of the
// workgroups already done: the flushes take the entry count from the low bits only.
#define GC_TICKET_SHIFT 40
#define GC_COUNT_MASK ((1ull << GC_TICKET_SHIFT) - 1ull)

// the bound of one wave's flush (base and count wave-uniform): false = overflow, reported
__device__ __forceinline__ bool gc_stage_fits(const GcStage& s, ull base) {
    if (base + (ull)s.cnt <= (ull)s.cap) return true;
    if (gc_lane() == 0) {
        __hip_atomic_store(s.err, GC_LERR_LIST, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(s.halt, GC_H_STALLED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return false;
}

__device__ __forceinline__ void gc_stage_flush(GcStage& s, int* out, ull* out_cnt) {
    gc_wave_sync();
    if (s.cnt == 0) return;
    ull base = 0;
    if (gc_lane() == 0) base = atomicAdd(out_cnt, (ull)s.cnt) & GC_COUNT_MASK;
    base = __shfl(base, 0, GC_WAVE);
    if (gc_stage_fits(s, base)) {
#pragma unroll 1
        for (int i = gc_lane(); i < s.cnt; i += GC_WAVE) out[base + i] = s.buf[i];
    }
    gc_wave_sync();
    s.cnt = 0;
}

// End-of-kernel flush for the whole workgroup (every thread calls): one global atomic per
// workgroup instead of one per wave -- thousands of waves each returning a handful of
// entries on one counter cost ~10 us per 1000 atomics.
template <int NW = GC_WAVES_PER_BLOCK>
__device__ __forceinline__ void gc_stage_flush_block(GcStage& s, int* out, ull* out_cnt) {
    __shared__ int s_cnt[NW];
    __shared__ ull s_base;
    const int w = threadIdx.x / GC_WAVE;
    gc_wave_sync();
    if (gc_lane() == 0) s_cnt[w] = s.cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int i = 0; i < NW; ++i) t += s_cnt[i];
        s_base = t ? atomicAdd(out_cnt, (ull)t) & GC_COUNT_MASK : 0ull;
    }
    __syncthreads();
    ull base = s_base;
    for (int i = 0; i < w; ++i) base += (ull)s_cnt[i];
    if (gc_stage_fits(s, base)) {
#pragma unroll 1
        for (int i = gc_lane(); i < s.cnt; i += GC_WAVE) out[base + i] = s.buf[i];
    }
    gc_wave_sync();
    s.cnt = 0;
    __syncthreads();
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

__device__ __forceinline__ long long gc_delta(int v, int val) {
    return (long long)(((ull)(unsigned)v << 32) | (ull)(unsigned)val);
}

// Wave-aggregated append of 64-bit entries.  All lanes must call.
__device__ __forceinline__ void gc_wave_append64(bool pred, long long val, long long* out, ull* out_cnt) {
    const ull m = __ballot(pred);
    if (m == 0) return;
    ull base = 0;
    const int leader = __ffsll((long long)m) - 1;
    if (gc_lane() == leader) base = atomicAdd(out_cnt, (ull)__popcll(m));
    base = __shfl(base, leader, GC_WAVE);
    if (pred) out[base + __popcll(m & gc_lanemask_lt())] = val;
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

// (reads first: the running max settles quickly, so most workgroups skip the atomic)
__device__ __forceinline__ void gc_block_max(long long* dst, long long v, long long* lds_scratch) {
    v = gc_wave_max(v);
    const int w = threadIdx.x / GC_WAVE;
    if (gc_lane() == 0) lds_scratch[w] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        long long t = lds_scratch[0];
        for (int i = 1; i < (int)(blockDim.x / GC_WAVE); ++i) t = lds_scratch[i] > t ? lds_scratch[i] : t;
        if (t >= 0 && t > __hip_atomic_load(dst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(dst, t);
    }
    __syncthreads();
}

__device__ __forceinline__ unsigned char gc_c8_of(long long c) {
    return c < 0 ? (unsigned char)GC_C8_NONE : (c >= 254 ? (unsigned char)GC_C8_BIG : (unsigned char)c);
}

// proposal byte k8 = cand6 << 2 | JP state; cand6 = candidate (< 62), GC_K8_BIG (>= 62:
// the candidate is in cand[]) or GC_K8_NONE (not proposing this round)
#define GC_K8_BIG 62u
#define GC_K8_NONE 63u
// hub mirror hk (one 32-bit word per hub): full candidate << 2 | JP state, so a hub JP
// step needs ONE gather per row entry (no separate candidate gather past colour 61)
#define GC_HK_COLOURED 0xFFFFFFFFu  // coloured
#define GC_HK_NOCAND 0x3FFFFFFEu    // candidate field of a hub that does not propose
__device__ __forceinline__ unsigned gc_hk(unsigned cand, unsigned st) { return (cand << 2) | st; }
__device__ __forceinline__ unsigned char gc_k8(unsigned c6, unsigned st) { return (unsigned char)((c6 << 2) | st); }
__device__ __forceinline__ unsigned gc_c6_of(long long c) { return c >= 62 ? GC_K8_BIG : (unsigned)c; }
__device__ __forceinline__ unsigned gc_k8_cand(unsigned k) { return k >> 2; }
__device__ __forceinline__ unsigned gc_k8_state(unsigned k) { return k & 3u; }

// The rank partition's first gather per entry (gc_prep.hip): a monotone byte code of the
// degree -- exact below 32, then 8 equal-width buckets per octave (d in [2^k, 2^(k+1)) ->
// 32 + 8 (k - 5) + floor(8 (d - 2^k) / 2^k), at most 239 for d < 2^31).  Different codes
// order two degrees; equal codes >= 32 need the degrees themselves.  Round 3 used min(deg,
// 255), so every entry between two vertices of degree >= 255 gathered the 4-byte degree too:
// 52% of R-MAT-22's entries, against 7% with this code (numpy R-MAT, tools-free count).
#define GC_DEG_CODE_EXACT 32u
__host__ __device__ __forceinline__ unsigned gc_deg_code(long long d) {
    if (d < (long long)GC_DEG_CODE_EXACT) return d < 0 ? 0u : (unsigned)d;
    const int lz = 63 - __builtin_clzll((ull)d);  // floor(log2 d) >= 5
    const ull rem = (ull)d - (1ull << lz);
    const unsigned c = GC_DEG_CODE_EXACT + 8u * (unsigned)(lz - 5) + (unsigned)((rem * 8ull) >> lz);
    return c < 255u ? c : 255u;
}

// rank order of coloring.py:64 (stable sort by deg of a file-ordered group): (deg, pos) asc
__device__ __forceinline__ bool gc_rank_lt(int du, int u, int dv, int v) {
    return du < dv || (du == dv && u < v);
}
// the same order over a 32-bit key (deg, or a seeded priority: gc_priority.hip)
__device__ __forceinline__ bool gc_rank_lt_key(unsigned ku, int u, unsigned kv, int v) {
    return ku < kv || (ku == kv && u < v);
}

// seeded 32-bit priority: the top half of splitmix64(seed + (v + 1) * golden gamma)
// (identical to prio_hash in oracle/gcolor_oracle.c)
__device__ __forceinline__ unsigned gc_prio_hash(ull seed, long long v) {
    ull z = seed + 0x9E3779B97F4A7C15ull * (ull)(v + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (unsigned)(z >> 32);
}
