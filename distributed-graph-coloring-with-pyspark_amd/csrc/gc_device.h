// gc_device.h -- device helpers shared by the kernel files (variant A rounds, variant B).
#pragma once
#include "gcolor.h"
#include "gc_internal.h"
#include "gc_launch.h"

// ------------------------------------------------------------------------------------
// chunk geometry shared by the light kernels
// ------------------------------------------------------------------------------------
__device__ __forceinline__ long long gc_nchunks(long long cnt, int vpw) { return (cnt + vpw - 1) / vpw; }

// Iterate the edge slots [0, total) of a wave chunk, GC_SLOTS 64-slot groups per step so
// each lane has GC_SLOTS independent col[] -> gather chains in flight (the waves spend most
// of their cycles waiting on these gathers).  load(u) returns the gathered value;
// apply(o, u, val, slot) consumes it for owner lane o (slot = offset in o's range).
#ifndef GC_SLOTS
#define GC_SLOTS 2
#endif
template <int SLOTS = GC_SLOTS, typename Load, typename Apply>
__device__ __forceinline__ void gc_chunk_edges_at(const int* __restrict__ col, const long long* s_start, int excl,
                                                  int total, Load load, Apply apply) {
    const int lane = gc_lane();
    for (int base = 0; base < total; base += SLOTS * GC_WAVE) {
        int o[SLOTS], x[SLOTS], u[SLOTS];
        bool ok[SLOTS];
#pragma unroll
        for (int k = 0; k < SLOTS; ++k) {
            const int e = base + k * GC_WAVE + lane;
            o[k] = gc_owner(excl, e);
            x[k] = e - __shfl(excl, o[k], GC_WAVE);
            ok[k] = e < total;
        }
#pragma unroll
        for (int k = 0; k < SLOTS; ++k) u[k] = ok[k] ? col[s_start[o[k]] + x[k]] : 0;
        decltype(load(0)) gv[SLOTS];
#pragma unroll
        for (int k = 0; k < SLOTS; ++k) gv[k] = ok[k] ? load(u[k]) : decltype(load(0)){};
#pragma unroll
        for (int k = 0; k < SLOTS; ++k)
            if (ok[k]) apply(o[k], u[k], gv[k], x[k]);
    }
}

template <int SLOTS = GC_SLOTS, typename Load, typename Apply>
__device__ __forceinline__ void gc_chunk_edges(const int* __restrict__ col, const long long* s_start, int excl,
                                               int total, Load load, Apply apply) {
    gc_chunk_edges_at<SLOTS>(col, s_start, excl, total, load,
                             [&](int o, int u, decltype(load(0)) v, int) { apply(o, u, v); });
}

// colour of u from the byte mirror (-1 uncoloured)
__device__ __forceinline__ int gc_colour(const GDev& g, int u) {
    const unsigned b = g.c8[u];
    return b == GC_C8_NONE ? -1 : (b == GC_C8_BIG ? g.color[u] : (int)b);
}

// Committed colours live in the byte mirror c8 (what propose gathers); the int32 colour
// array is written only for colours >= 254 and rebuilt from c8 by k_finalize.
__device__ __forceinline__ void gc_commit_colour(GDev& g, int v, int cc) {
    const unsigned char b = gc_c8_of(cc);
    g.c8[v] = b;
    if (b == GC_C8_BIG) g.color[v] = cc;
    g.k8[v] = (unsigned char)gc_k8(GC_K8_NONE, GC_JP_UND);
    if (g.hub_w) {  // hub mirror (gc_hubs.hip)
        const int x = g.hid[v];
        if (x >= 0) g.hk[x] = GC_HK_COLOURED;
    }
}

// the same without resetting k8 (fused commit, k_commit<1>: the winner's IN byte stays, so
// waves proposing for the next round see its colour before its c8 byte lands)
__device__ __forceinline__ void gc_commit_colour_keep(GDev& g, int v, int cc) {
    const unsigned char b = gc_c8_of(cc);
    g.c8[v] = b;
    if (b == GC_C8_BIG) g.color[v] = cc;
}

// counters shared across workgroups: read with an atomic RMW, written agent-scope
__device__ __forceinline__ ull gc_aread(ull* p) { return atomicAdd(p, 0ull); }
template <typename T>  // (host too: tests/host_close runs the round close on the CPU)
__host__ __device__ __forceinline__ void gc_st(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Word t of hub x's forbidden-colour bitmap.  GC_HB_WMAJOR=1 (round 6, measured and left off):
// words stored word-major -- word t of every hub together -- so that the words a round touches
// (its newest colours' word) are a few hundred KB; R-MAT-24 +5 ms, R-MAT-26 +1.3 ms against
// the hub-major rows (profiles/r06/u): a big round's proposals read several words per hub.
#ifndef GC_HB_WMAJOR
#define GC_HB_WMAJOR 0
#endif
__device__ __forceinline__ unsigned* gc_hbw(const GDev& g, long long x, long long t) {
#if GC_HB_WMAJOR
    return g.hbits + t * g.hb_stride + x;
#else
    return g.hbits + x * g.hbits_w + t;
#endif
}
// hubs (gc_hubs.hip): set colour cc in hub x's forbidden-colour bitmap (colours past the
// bitmap are not tracked: such a hub scans its row when its mex could lie beyond it)
__device__ __forceinline__ void gc_hub_mark(const GDev& g, int x, int cc) {
    if (g.hseen && !g.hseen[x]) g.hseen[x] = 1;  // shards: the hub now belongs to a frontier
    if (cc >= 32 * g.hbits_w) return;
    unsigned* p = gc_hbw(g, x, cc >> 5);
    const unsigned bit = 1u << (cc & 31);
    if (!(*p & bit)) atomicOr(p, bit);
}
// every hub listing v, strided over the calling threads
__device__ __forceinline__ void gc_hub_mark_row(const GDev& g, int v, int cc, int t0, int step) {
    const long long e1 = g.hin_rp[v + 1];
    for (long long e = g.hin_rp[v] + t0; e < e1; e += step) gc_hub_mark(g, g.hin_col[e], cc);
}
// the marks of a wave's flat range [0, total) of hub entries; entry(e, &x, &cc) gives entry
// e's hub index and colour (all 64 lanes call it: it may shuffle; x = -1 past total)
// (round 3's GC_MARK_SLOTS=4 -- four entries per thread and step, loads before the atomics --
// measured within noise on R-MAT-24 in round 4, 171.3-171.9 vs 171.2-173.5 ms, profiles/r04/c:
// removed, with GC_CLAIM_HOIST and GC_HIN_HOIST)
template <typename Entry>
__device__ __forceinline__ void gc_hub_mark_flat(const GDev& g, int total, Entry entry) {
    const int lane = gc_lane();
    for (int base = 0; base < total; base += GC_WAVE) {
        int x, c;
        entry(base + lane, &x, &c);
        if (x >= 0) gc_hub_mark(g, x, c);
    }
}
// Pushes of this wave's winners' colours into the hub bitmaps (hbits_w), the wave walking
// its lanes' hub lists as one flat range; a list longer than GC_PUSH_FLAT is appended to
// `big` for gcl_hub_push_big (a workgroup each: one thread per winner walked lists of
// thousands).  All 64 lanes call; s_start / s_cc are this wave's LDS rows.
#define GC_PUSH_FLAT 256
__device__ __forceinline__ void gc_hub_push_wave(const GDev& g, bool win, int v, int cc, long long* s_start, int* s_cc,
                                                 int* big, ull* big_cnt) {
    const int lane = gc_lane();
    long long hs = 0;
    int hl = 0;
    if (win) {
        hs = g.hin_rp[v];
        hl = (int)(g.hin_rp[v + 1] - hs);
    }
    const bool far = hl > GC_PUSH_FLAT;
    gc_wave_append(far, v, big, big_cnt);
    if (far) hl = 0;
    s_start[lane] = hs;
    s_cc[lane] = cc;
    const int incl = gc_wave_incl_scan(hl);
    const int excl = incl - hl;
    const int total = __shfl(incl, GC_WAVE - 1, GC_WAVE);
    gc_wave_sync();
    gc_hub_mark_flat(g, total, [&](int e, int* x, int* c) {
        const int o = gc_owner(excl, e);
        const int eo = __shfl(excl, o, GC_WAVE);
        *x = e < total ? g.hin_col[s_start[o] + (e - eo)] : -1;
        *c = e < total ? s_cc[o] : 0;
    });
    gc_wave_sync();
}

// agent-scope (sc1) loads and stores of state another workgroup of the same launch reads or
// writes (the asynchronous JP, k_sweep_async; variant B's asynchronous fold): stores write
// through past this XCD's L2, loads bypass L1
__device__ __forceinline__ unsigned gc_ald8(const unsigned char* p) {
    return (unsigned)__hip_atomic_load(const_cast<unsigned char*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned gc_ald32(const unsigned* p) {
    return __hip_atomic_load(const_cast<unsigned*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int gc_aldi(const int* p) {
    return __hip_atomic_load(const_cast<int*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gc_ast8(unsigned char* p, unsigned v) {
    __hip_atomic_store(p, (unsigned char)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gc_ast32(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gc_asti(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// heavy entries the one-workgroup tail sweeps may take
__device__ __forceinline__ long long gc_tail_hmax(const GDev& g) { return g.tail_hmax; }

// Which hubs sweep i (>= 1) takes, from values fixed before the kernel (gc_hubs.hip): hubs
// off -- the undecided heavy list; hubs already started (hub_start < i) -- likewise; not
// started and the lights converged (cl == 0) -- every hub proposer, and this sweep starts
// them (returns true: the caller records hub_start = i); lights still undecided -- none.
// The caller's thread 0 may store hub_start = i while other workgroups evaluate this: they
// read either the old value (>= i) or i, and take the same branch either way.
__device__ __forceinline__ bool gc_hub_gate(const GDev& g, const DevCtl* c, long long i, long long cl,
                                            const int*& hl, long long& ch, const GLists& L) {
    if (!g.hub_w || __hip_atomic_load(const_cast<long long*>(&c->hub_start), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < i) return false;
    if (cl == 0 && !c->lights_hold) {  // shards: every rank's lights (gc_shard_release_hubs)
        hl = L.heavy;
        ch = (long long)c->heavy_cnt;
        return true;
    }
    ch = 0;
    return false;
}

// Algorithmic-byte counters (stats only): a workgroup adds into slot blockIdx % GC_STAT_SLOTS
// instead of every workgroup hitting the same two DevCtl words; k_stat_reduce sums them.
#ifndef GC_STAT_WAVE
#define GC_STAT_WAVE 1  // measured: R-MAT-24 226 vs 228 ms with the per-workgroup reduction
#endif
template <int NW = GC_WAVES_PER_BLOCK>
__device__ __forceinline__ void gc_stat_add(const GDev& g, int cls, ull lsum, ull lnv, ull* lds_scratch) {
    lsum = gc_wave_sum(lsum);
    lnv = gc_wave_sum(lnv);
#if GC_STAT_WAVE  // each wave adds its own sums (no workgroup barriers at the kernel's end)
    (void)lds_scratch;
    if (gc_lane() == 0) {
        ull* slot = g.bstat + ((blockIdx.x * NW + threadIdx.x / GC_WAVE) % GC_STAT_SLOTS) * 16;
        if (lsum) atomicAdd(slot + cls, lsum);
        if (lnv) atomicAdd(slot + 8 + cls, lnv);
    }
    return;
#endif
    const int w = threadIdx.x / GC_WAVE;
    if (gc_lane() == 0) {
        lds_scratch[w] = lsum;
        lds_scratch[NW + w] = lnv;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        ull a = 0, b = 0;
        for (int i = 0; i < (int)(blockDim.x / GC_WAVE); ++i) {
            a += lds_scratch[i];
            b += lds_scratch[NW + i];
        }
        ull* slot = g.bstat + (blockIdx.x % GC_STAT_SLOTS) * 16;
        if (a) atomicAdd(slot + cls, a);
        if (b) atomicAdd(slot + 8 + cls, b);
    }
    __syncthreads();
}

// Residency probe (budget < 0 in k_sweep_async / k_b_async: the SAME kernel, so the same
// registers, SGPRs and LDS): lane 0 of every workgroup arrives on c->async_done[0] and waits
// until every workgroup of the grid has arrived or ~100 us have passed; the first to leave
// records the arrivals it saw in c->async_done[1].  Resident workgroups all start at once and
// none leaves before the wait ends, so that record is the number that fit on the device at
// once -- what the asynchronous kernels' static slices need (gc_resident_blocks_per_cu's
// runtime query cannot see SGPR limits: k_b_async's 106 SGPRs allow 7 waves per SIMD where the
// runtime answered 8).
__device__ __forceinline__ void gc_residency_probe(DevCtl* c) {
    if (threadIdx.x != 0) return;
    atomicAdd(&c->async_done[0], 1ull);
    const ull t0 = wall_clock64();
    ull v = 0;
    for (;;) {
        v = __hip_atomic_load(&c->async_done[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v >= (ull)gridDim.x || wall_clock64() - t0 > 10000) break;  // 100 MHz: 100 us
        __builtin_amdgcn_s_sleep(4);
    }
    atomicCAS(&c->async_done[1], 0ull, v);
}
