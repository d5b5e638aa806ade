// gc_kernels.hip -- gfx950 kernels of the colouring round (variant A, coloring.py:73-132).
//
// The round is a fixed sequence of launches that the host enqueues WITHOUT reading
// anything back: every kernel takes its work counts from the device control block
// (DevCtl), runs a fixed grid that grid-strides over them, and returns at once when a
// previous kernel raised DevCtl.halt.  Per round r:
//   k_propose       mex of coloured neighbours' colours, colours as at the round start
//                   (coloring.py:44-54, 82-83, 98-102); gathers the 1-byte colour mirror
//   k_propose_block hubs (deg > GC_HEAVY_T) and light vertices whose mex >= 64
//   k_resolve       first Jones-Plassmann sweep of the per-candidate-colour conflict
//                   resolution: the lexicographically-first maximal independent set under
//                   rank (deg asc, pos asc) == coloring.py:56-70's stable-sorted greedy
//                   pass; raises GC_H_FAILED for a bounded attempt (coloring.py:104-108)
//   k_sweep x S     further JP sweeps over the undecided lists (rotating slots)
//   k_commit        scatter accepted colours (coloring.py:37-41, 114-127), push the next
//                   frontier through the in-neighbour lists (claim bitmap + LDS-staged
//                   appends); its last workgroup closes the round: per-round record,
//                   counter reset, termination / E1 / "more sweeps" decisions.
// E1 re-seed (k_unc_compact, k_cc_hook, k_cc_best, k_cc_seeds) and the validator
// (k_validate, coloring.py:149-162) live here too.
//
// Edge-balanced wave chunks: a wave takes `vpw` list entries (64 for big lists, fewer for
// short ones), prefix-sums their degrees and walks the concatenated edge range 64 slots
// at a time (two slots in flight per lane), so consecutive lanes read consecutive col[]
// entries and no lane idles on a short row.  All of it is HBM/L2-bound gather work; no
// MFMA involved.
#include <stdlib.h>

#include <algorithm>

#include <map>
#include <mutex>

#include "gcolor.h"
#include "gc_internal.h"
#include "gc_launch.h"
#include "gc_device.h"
#include "gc_close.h"



// ------------------------------------------------------------------------------------
// init: coloring.py:12-17 (+ argmax seed key for coloring.py:19-35)
// ------------------------------------------------------------------------------------
// Isolated vertices are coloured at init; when some OTHER vertex lists one of them
// (asymmetric input) it must push like a committed vertex, so it joins the seed list.
__global__ void __launch_bounds__(GC_BLOCK) k_init(GDev g, int* seed_light) {
    __shared__ ull scratch[2 * GC_WAVES_PER_BLOCK];
    const int lane = gc_lane();
    ull best = 0, unc = 0;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v - lane < g.n; v += stride) {
        const bool valid = v < g.n;
        const int d = valid ? g.deg[v] : 0;
        const bool iso = valid && d == 0;
        // (replicated hubs, gc_shard.hip: also when a hub lists it, so every rank marks that hub)
        const bool push0 = iso && (g.trp[v + 1] > g.trp[v] || (g.hub_repl && g.hin_rp[v + 1] > g.hin_rp[v]));
        if (valid) {
            g.color[v] = iso ? 0 : -1;
            g.cround[v] = iso ? 0 : -1;
            g.c8[v] = iso ? 0 : (unsigned char)GC_C8_NONE;
            g.k8[v] = push0 ? gc_k8(0u, GC_JP_IN) : gc_k8(GC_K8_NONE, GC_JP_UND);
            if (g.hub_w && g.hid[v] >= 0)  // hub mirror (never isolated)
                g.hk[g.hid[v]] = gc_hk(GC_HK_NOCAND, GC_JP_UND);
            g.mark[v] = 0;
            if (!iso) {
                unc++;
                const ull k = ((ull)d << 32) | (ull)v;
                best = k > best ? k : best;
            }
        }
        gc_wave_append(push0, (int)v, seed_light, &g.ctl->seed_cnt[0]);
        // claim bitmap: isolated vertices are coloured (never enter a frontier)
        const ull m = __ballot(iso || !valid);
        if (lane == 0) {
            const long long w = (v - lane) >> 5;
            g.inF[w] = (unsigned)m;
            if ((v - lane) + 32 < g.n) g.inF[w + 1] = (unsigned)(m >> 32);
        }
    }
    // seed argmax: max (deg << 32 | pos) == last max-degree vertex in file order
    best = gc_wave_max(best);
    const int w = threadIdx.x / GC_WAVE;
    if (lane == 0) scratch[w] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        ull t = 0;
        for (int i = 0; i < GC_WAVES_PER_BLOCK; ++i) t = scratch[i] > t ? scratch[i] : t;
        if (t) atomicMax(&g.ctl->seedkey, t);
    }
    __syncthreads();
    gc_block_add(&g.ctl->uncolored, unc, scratch);
}

// Prepare the seed chosen by k_init as an accepted colour-0 vertex (coloring.py:25).
__global__ void k_seed_prep(GDev g, int* seed_light, int* seed_heavy) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const ull sk = g.ctl->seedkey;
    if (sk == 0) return;
    const int s = (int)(sk & 0xFFFFFFFFull);
    const int d = g.deg[s];
    g.k8[s] = gc_k8(0u, GC_JP_IN);
    if (g.hub_w && g.hid[s] >= 0) g.hk[g.hid[s]] = gc_hk(0u, GC_JP_IN);
    atomicOr(&g.inF[s >> 5], 1u << (s & 31));
    if (d > GC_HEAVY_T) seed_heavy[atomicAdd(&g.ctl->seed_cnt[1], 1ull)] = s;
    else seed_light[atomicAdd(&g.ctl->seed_cnt[0], 1ull)] = s;
}

// ------------------------------------------------------------------------------------
// Frontier re-sort for big rounds.  The frontier list is built by appends (losers and
// newly claimed vertices in arrival order), so the per-vertex metadata reads of propose /
// resolve / commit would be random.  When the frontier is large (>= n/64) it is rebuilt
// in vertex order from the bitmaps -- frontier == claimed (inF) and still uncoloured (c8)
// -- in three passes over n/32 words: per-workgroup counts, one-workgroup scan, ordered
// write.  Same set, same count; the order is irrelevant to the results.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned gc_front_word(const GDev& g, long long w) {
    const unsigned m = g.inF[w];
    if (!m) return 0u;
    const long long v0 = w * 32;
    unsigned out = 0u;
    if (v0 + 32 <= (long long)g.n) {
        const uint4* p = reinterpret_cast<const uint4*>(g.c8 + v0);
        const uint4 a = p[0], b = p[1];
        const unsigned x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            // bytes equal to 0xFF (uncoloured): zero bytes of ~x, exact per byte
            const unsigned t = ~x[k];
            const unsigned z = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);  // 0x80 where byte == 0
            const unsigned nib = ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
            out |= nib << (4 * k);
        }
    } else {
        for (int k = 0; k < 32 && v0 + k < (long long)g.n; ++k)
            if (g.c8[v0 + k] == GC_C8_NONE) out |= 1u << k;
    }
    return out & m;
}


__global__ void __launch_bounds__(GC_BLOCK) k_fsort_count(GDev g, unsigned* bsum) {
    DevCtl* c = g.ctl;
    if (c->halt) return;
    // fsort_all: list = every claimed uncoloured vertex; a list built by k_front_* is in order already
    const bool on = c->fsort_all ? true : (gc_resort_on(g, c) && !c->sorted);
    if (blockIdx.x == 0 && threadIdx.x == 0) c->resort = on ? 1 : 0;
    if (!on) return;
    __shared__ ull scratch[2 * GC_WAVES_PER_BLOCK];
    const long long words = ((long long)g.n + 31) / 32;
    const long long w = (long long)blockIdx.x * GC_BLOCK + threadIdx.x;
    ull cnt = w < words ? (ull)__popc(gc_front_word(g, w)) : 0ull;
    cnt = gc_wave_sum(cnt);
    if (gc_lane() == 0) scratch[threadIdx.x / GC_WAVE] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        ull t = 0;
        for (int i = 0; i < GC_WAVES_PER_BLOCK; ++i) t += scratch[i];
        bsum[blockIdx.x] = (unsigned)t;
    }
}

// exclusive scan of the per-workgroup counts, one workgroup of 1024 threads
// build = 0: the re-sort of the current list; build = 1: the next frontier of a big round
// (k_front_count), whose total becomes its count.
__global__ void __launch_bounds__(1024) k_fsort_scan(GDev g, unsigned* bsum, int nblocks, int build) {
    DevCtl* c = g.ctl;
    if (build ? !gc_front_on(g, c, 1) : (c->halt || !c->resort)) return;
    __shared__ unsigned s_part[1024];
    const int per = (nblocks + 1023) / 1024;
    const int b0 = threadIdx.x * per;
    unsigned local = 0;
    for (int i = 0; i < per && b0 + i < nblocks; ++i) local += bsum[b0 + i];
    s_part[threadIdx.x] = local;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
        const unsigned y = threadIdx.x >= off ? s_part[threadIdx.x - off] : 0u;
        __syncthreads();
        s_part[threadIdx.x] += y;
        __syncthreads();
    }
    if (threadIdx.x == 1023) {
        if (build) c->fcnt[c->cur ^ 1] = s_part[1023];
        else if (c->fsort_all) c->fcnt[c->cur] = s_part[1023];  // the list is rebuilt, not re-sorted
    }
    unsigned run = s_part[threadIdx.x] - local;  // exclusive prefix of this thread's run
    for (int i = 0; i < per && b0 + i < nblocks; ++i) {
        const unsigned x = bsum[b0 + i];
        bsum[b0 + i] = run;
        run += x;
    }
}

__global__ void __launch_bounds__(GC_BLOCK) k_fsort_write(GDev g, const unsigned* bpre, GLists L, int build) {
    DevCtl* c = g.ctl;
    if (build ? !gc_front_on(g, c, 1) : (c->halt || !c->resort)) return;
    __shared__ unsigned s_w[GC_WAVES_PER_BLOCK];
    const long long words = ((long long)g.n + 31) / 32;
    const long long w = (long long)blockIdx.x * GC_BLOCK + threadIdx.x;
    const unsigned m = w < words ? gc_front_word(g, w) : 0u;
    const int cnt = __popc(m);
    const int incl = gc_wave_incl_scan(cnt);
    if (gc_lane() == GC_WAVE - 1) s_w[threadIdx.x / GC_WAVE] = (unsigned)incl;
    __syncthreads();
    unsigned off = bpre[blockIdx.x];
    for (int i = 0; i < (int)(threadIdx.x / GC_WAVE); ++i) off += s_w[i];
    off += (unsigned)(incl - cnt);
    int* out = L.F[build ? c->cur ^ 1 : c->cur];
    unsigned mm = m;
    while (mm) {
        const int k = __builtin_ctz(mm);
        mm &= mm - 1u;
        out[off++] = (int)(w * 32 + k);
    }
}

// ------------------------------------------------------------------------------------
// nibble colour mirror for the big rounds of few-colour graphs: 8 vertices per word
// (half the footprint of c8 against the 4 MB L2 per XCD).  Built when the frontier is
// large (>= n/32) and every committed colour is < 14, else the round gathers c8.
// ------------------------------------------------------------------------------------
__global__ void __launch_bounds__(GC_BLOCK) k_pack_c4(GDev g) {
    DevCtl* c = g.ctl;
    if (c->halt) return;
    const long long words = ((long long)g.n + 7) >> 3;
    const bool on = (long long)c->fcnt[c->cur] * 32 >= (long long)g.n && c->maxcolor < 14;
    if (blockIdx.x == 0 && threadIdx.x == 0) c->use_c4 = on ? 1 : 0;
    if (!on) return;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < words;
         i += (long long)gridDim.x * blockDim.x) {
        unsigned lo = 0xFFFFFFFFu, hi = 0xFFFFFFFFu;
        if (8 * i + 8 <= g.n) {
            const uint2 b = *reinterpret_cast<const uint2*>(g.c8 + 8 * i);
            lo = b.x;
            hi = b.y;
        } else {
            unsigned char t[8];
            for (int k = 0; k < 8; ++k) t[k] = 8 * i + k < g.n ? g.c8[8 * i + k] : 0xFF;
            lo = t[0] | (t[1] << 8) | (t[2] << 16) | ((unsigned)t[3] << 24);
            hi = t[4] | (t[5] << 8) | (t[6] << 16) | ((unsigned)t[7] << 24);
        }
        unsigned wv = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const unsigned a = (lo >> (8 * k)) & 0xFFu, b = (hi >> (8 * k)) & 0xFFu;
            wv |= (a < 14u ? a : 15u) << (4 * k);
            wv |= (b < 14u ? b : 15u) << (4 * (k + 4));
        }
        g.c4[i] = wv;
    }
}

// ------------------------------------------------------------------------------------
// propose (assign_color, coloring.py:44-54)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void gc_set_cand(GDev& g, int v, long long mex) {
    const unsigned c6 = gc_c6_of(mex);
    if (c6 == GC_K8_BIG) g.cand[v] = (int)mex;
    g.k8[v] = gc_k8(c6, GC_JP_UND);
}

// INL = 1 (the one-GPU engine's small rounds, GC_INLINE_PB): the heavy proposers (hubs, whose
// forbidden colours are pushed bitmaps covering every colour in use) and the wide lights
// (mex >= 64, so mex <= deg <= heavy_t < GC_INL_BITS) are proposed here, the whole wave on
// one of them at a time, instead of in a k_propose_block launch after this one.
#define GC_INL_WORDS 32  // 2048-bit LDS window per wave for a wide light's mex
#ifndef GC_PH_B
#define GC_PH_B 4  // hub bitmaps read together by k_propose<1>
#endif
#define GC_INL_BITS (64 * GC_INL_WORDS)
#ifndef GC_PROP_STAGE
#define GC_PROP_STAGE 1  // k_propose: heavy-list appends staged per workgroup (round 6)
#endif
#ifndef GC_VPW_MIN_P
#define GC_VPW_MIN_P 16  // k_propose<1> (small rounds): vertices per wave chunk at least (round 6)
#endif
#ifndef GC_PROP_HINT
#define GC_PROP_HINT 1  // k_propose<1>: hub bitmaps read from the last proposal's word (round 6)
#endif
#ifndef GC_HOIST_HIN
#define GC_HOIST_HIN 0  // light kernels: cand / hin_rp loaded with the vertex's other words (round 6;
                        // measured slower: the big rounds' extra loads, R-MAT-26 +3.6 ms, profiles/r06/q)
#endif
#ifndef GC_PB_HUB_LANES
#define GC_PB_HUB_LANES 1  // k_propose_block: a run of hubs per wave, one per lane (round 6)
#endif
template <int INL>
__global__ void __launch_bounds__(GC_BLOCK) k_propose(GDev g, GLists L) {
    DevCtl* c = g.ctl;
    if (c->halt) return;
    __shared__ ull s_mask[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ ull s_wide[INL ? GC_WAVES_PER_BLOCK : 1][INL ? GC_INL_WORDS : 1];
    __shared__ long long s_start[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ ull scratch[2 * GC_WAVES_PER_BLOCK];
#if GC_PROP_STAGE
    // the heavy list's appends staged in LDS, one atomic per workgroup at the end (round 6): a
    // returning atomic per wave on the one counter cost ~11 ns each, serialised -- ~1500 waves
    // with a hub in a 12k-vertex round, most of k_propose's 20 us
    __shared__ int s_hstage[GC_WAVES_PER_BLOCK][GC_STAGE_CAP];
#endif
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    const int cur = c->cur;
    const int* __restrict__ list = L.F[cur];
    const long long cnt = (long long)c->fcnt[cur];
    const long long kbound = c->kbound;
    int vpw = gc_vpw(cnt, (long long)gridDim.x * GC_WAVES_PER_BLOCK);
    // small rounds: at least GC_VPW_MIN_P vertices a wave chunk, so fewer waves and workgroups
    // take part (each one's appends cost an atomic on a shared counter; round 6)
    if (INL && vpw < GC_VPW_MIN_P) vpw = GC_VPW_MIN_P;
#if GC_PROP_STAGE
    GcStage hst{s_hstage[w], 0, g.list_cap, &c->loop_err, &c->halt};
#endif
    const long long nch = gc_nchunks(cnt, vpw);
    long long lmax = -1;
    ull lfail = 0, lsum = 0, lnv = 0;
    const unsigned char* __restrict__ c8 = g.c8;
    const unsigned* __restrict__ c4 = g.c4;
    const bool use_c4 = c->use_c4 != 0;
    long long hwords = INL ? (c->maxcolor + 2 + 31) / 32 : 0;  // the bitmap words in use (mex <= maxcolor + 1)
    if (INL && hwords > g.hbits_w) {  // the host's margin was too small: report, propose nothing
        if (threadIdx.x == 0 && blockIdx.x == 0)
            __hip_atomic_store(&c->loop_err, GC_LERR_INL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    for (long long ch = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w; ch < nch;
         ch += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
        const long long idx = ch * vpw + lane;
        const int v = (lane < vpw && idx < cnt) ? list[idx] : -1;
        const int d = v >= 0 ? g.deg[v] : 0;
        const bool isheavy = d > g.heavy_t;
#if GC_PROP_STAGE
        gc_stage_push(hst, isheavy, v, L.heavy, &c->heavy_cnt);
#else
        gc_wave_append(isheavy, v, L.heavy, &c->heavy_cnt);
#endif
        if (g.hub_repl) {  // replicated hubs of other ranks: in this rank's lists, not in its F
            const ull xm = __ballot(isheavy && (v < g.own_lo || v >= g.own_hi));
            if (xm && gc_lane() == 0) atomicAdd(&c->xhub_cnt, (ull)__popcll(xm));
        }
        const int de = isheavy ? 0 : d;
        s_mask[w][lane] = 0;
        s_start[w][lane] = v >= 0 ? g.rp[v] : 0;
        // GC_PROP_HINT (round 6): a hub's bitmap is read from the word of its last proposal on:
        // bits are only ever set, so the mex never moves down, and a hub proposes about the
        // newest colour every round (the first ~maxcolor/32 words are full).  The hint comes
        // from its own k8 / cand words, loaded with its degree, and the two words from it are
        // in flight with the light rows' loads: no dependent trip of its own.
        int hx = -1, hw0 = 0;
        unsigned hwa = 0xFFFFFFFFu, hwb = 0xFFFFFFFFu;
        if (INL && GC_PROP_HINT) {
            const int xs = v >= 0 ? g.hid[v] : -1;
            const unsigned k8v = v >= 0 ? (unsigned)g.k8[v] : 0u;
            const int cbv = v >= 0 ? g.cand[v] : 0;
            if (isheavy && xs >= 0) {
                hx = xs;
                const unsigned c6 = gc_k8_cand(k8v);
                const long long hint = c6 == GC_K8_NONE ? 0ll : (c6 == GC_K8_BIG ? (long long)cbv : (long long)c6);
                hw0 = (int)(hint >> 5);
                if (hw0 < 0 || hw0 >= hwords) hw0 = 0;
                hwa = *gc_hbw(g, hx, hw0);
                if (hw0 + 1 < hwords) hwb = *gc_hbw(g, hx, hw0 + 1);
            }
        }
        const int incl = gc_wave_incl_scan(de);
        const int excl = incl - de;
        const int total = __shfl(incl, GC_WAVE - 1, GC_WAVE);
        gc_wave_sync();
        if (use_c4) {  // nibble mirror: 0..13 colour, 14 never (maxcolor < 14), 15 uncoloured
            gc_chunk_edges(
                g.col, s_start[w], excl, total, [&](int u) { return (c4[u >> 3] >> ((u & 7) * 4)) & 15u; },
                [&](int o, int, unsigned cc) {
                    if (cc < 15u) atomicOr(&s_mask[w][o], 1ull << cc);
                });
        } else {
            gc_chunk_edges(
                g.col, s_start[w], excl, total, [&](int u) { return (unsigned)c8[u]; },
                [&](int o, int, unsigned cc) {
                    if (cc < 64u) atomicOr(&s_mask[w][o], 1ull << cc);
                });
        }
        gc_wave_sync();
        bool iswide = false;
        if (v >= 0 && !isheavy) {
            const ull m = s_mask[w][lane];
            if (m == ~0ull) {
                iswide = true;
            } else {
                const int mex = __builtin_ctzll(~m);
                gc_set_cand(g, v, mex);
                lmax = mex > lmax ? mex : lmax;
                if (kbound >= 0 && mex >= kbound) lfail++;
                lsum += (ull)d;
                lnv++;
            }
        }
        if (!INL) {
            gc_wave_append(iswide, v, L.wide, &c->wide_cnt);
            continue;
        }
        // hubs: the first zero bit of the pushed bitmap (as k_propose_block's hub waves), the
        // whole wave on each bitmap's words; the chunk's hub indices are loaded one per lane and
        // GC_PH_B bitmaps are read together, so a chunk of h hubs costs 1 + h / GC_PH_B
        // dependent trips (a hub at a time: 2 h), and every hub's own state is written by its
        // lane, all at once
        if (GC_PROP_HINT && hx >= 0) {  // the first zero bit from the hint's word on
            long long mex = -1;
            if (hwa != 0xFFFFFFFFu) {
                mex = 32ll * hw0 + __builtin_ctz(~hwa);
            } else if (hwb != 0xFFFFFFFFu) {
                mex = 32ll * (hw0 + 1) + __builtin_ctz(~hwb);
            } else {
                for (int t = hw0 + 2; t < hwords && mex < 0; ++t) {
                    const unsigned wd = *gc_hbw(g, hx, t);
                    if (wd != 0xFFFFFFFFu) mex = 32ll * t + __builtin_ctz(~wd);
                }
            }
            if (g.hub_w) {  // the hub JP's state: this round's conflict flag, cursors, mirror
                g.hkill[hx] = 0u;
                g.hcur[hx] = 0;
                g.hpc[hx] = 0;
                if (g.hprep) g.hkcnt[hx] = 0;
                g.hk[hx] = gc_hk((unsigned)mex, GC_JP_UND);
            }
            gc_set_cand(g, v, mex);
            lmax = mex > lmax ? mex : lmax;
            if (kbound >= 0 && mex >= kbound) lfail++;
            lsum += (ull)d;
            lnv++;
        }
        if (const ull hm0 = GC_PROP_HINT ? 0ull : __ballot(isheavy)) {
            const int xl = isheavy ? g.hid[v] : -1;
            long long hmex = -1;  // this lane's hub's mex
            for (ull hm = hm0; hm;) {
                int hl[GC_PH_B];
                int hbx[GC_PH_B];
                long long mx[GC_PH_B];
#pragma unroll
                for (int k = 0; k < GC_PH_B; ++k) {
                    hl[k] = hm ? __ffsll((long long)hm) - 1 : -1;  // wave-uniform
                    hm &= hm - 1;
                    const int xk = __shfl(xl, hl[k] < 0 ? 0 : hl[k], GC_WAVE);
                    hbx[k] = hl[k] < 0 ? 0 : xk;
                    mx[k] = hl[k] < 0 ? 0 : -1;
                }
                for (int t0 = 0; t0 < hwords; t0 += GC_WAVE) {  // a zero bit lies in range
                    const int t = t0 + lane;
                    unsigned wd[GC_PH_B];
#pragma unroll
                    for (int k = 0; k < GC_PH_B; ++k) wd[k] = (mx[k] < 0 && t < hwords) ? *gc_hbw(g, hbx[k], t) : 0xFFFFFFFFu;
                    bool done = true;
#pragma unroll
                    for (int k = 0; k < GC_PH_B; ++k) {
                        const ull zm = __ballot(wd[k] != 0xFFFFFFFFu);
                        if (mx[k] < 0 && zm) {
                            const int zl = __ffsll((long long)zm) - 1;
                            const unsigned zw = __shfl(wd[k], zl, GC_WAVE);
                            mx[k] = 32ll * (t0 + zl) + __builtin_ctz(~zw);
                        }
                        done = done && mx[k] >= 0;
                    }
                    if (done) break;
                }
#pragma unroll
                for (int k = 0; k < GC_PH_B; ++k)
                    if (lane == hl[k]) hmex = mx[k];
            }
            if (isheavy) {
                const int x = xl;
                const long long mex = hmex;
                if (g.hub_w) {  // the hub JP's state: this round's conflict flag, cursors, mirror
                    g.hkill[x] = 0u;
                    g.hcur[x] = 0;
                    g.hpc[x] = 0;
                    if (g.hprep) g.hkcnt[x] = 0;
                    g.hk[x] = gc_hk((unsigned)mex, GC_JP_UND);
                }
                gc_set_cand(g, v, mex);
                lmax = mex > lmax ? mex : lmax;
                if (kbound >= 0 && mex >= kbound) lfail++;
                lsum += (ull)d;
                lnv++;
            }
        }
        // wide lights: mex <= deg < GC_INL_BITS, one pass over the row into an LDS window
        for (ull wm = __ballot(iswide); wm; wm &= wm - 1) {
            const int l = __ffsll((long long)wm) - 1;
            const int wv = __shfl(v, l, GC_WAVE);
            const int wdg = __shfl(d, l, GC_WAVE);
            const long long rs = s_start[w][l];
            if (lane < GC_INL_WORDS) s_wide[w][lane] = 0ull;
            gc_wave_sync();
            for (int e = lane; e < wdg; e += GC_WAVE) {
                const int cc = gc_colour(g, g.col[rs + e]);
                if (cc >= 0 && cc < GC_INL_BITS) atomicOr(&s_wide[w][cc >> 6], 1ull << (cc & 63));
            }
            gc_wave_sync();
            const ull wk = lane < GC_INL_WORDS ? s_wide[w][lane] : ~0ull;
            const ull zm = __ballot(wk != ~0ull);  // nonzero: at most deg colours are forbidden
            const int zk = __ffsll((long long)zm) - 1;
            const ull zw = __shfl(wk, zk, GC_WAVE);
            const int mex = 64 * zk + __builtin_ctzll(~zw);
            if (lane == 0) {
                gc_set_cand(g, wv, mex);
                lmax = mex > lmax ? mex : lmax;
                if (kbound >= 0 && mex >= kbound) lfail++;
                lsum += (ull)wdg;
                lnv++;
            }
            gc_wave_sync();
        }
    }
#if GC_PROP_STAGE
    gc_stage_flush_block(hst, L.heavy, &c->heavy_cnt);
#endif
    __syncthreads();
    gc_block_max(&c->maxmex, lmax, (long long*)scratch);
    gc_block_add(&c->failcnt, lfail, scratch);
    gc_stat_add(g, GC_K_PROPOSE, lsum, lnv, scratch);
}

// One workgroup per vertex: hubs (deg > GC_HEAVY_T) and light vertices whose mex >= 64.
// Forbidden-colour bitmap in LDS covering [base, base + 32*GC_MEX_WORDS); mex <=
// maxcolor + 1, so one window suffices unless the colour count outgrows it.
__global__ void __launch_bounds__(GC_BLOCK) k_propose_block(GDev g, GLists L) {
    DevCtl* c = g.ctl;
    if (c->halt) return;
    extern __shared__ __attribute__((aligned(16))) unsigned s_bits[];
    __shared__ int s_first;
    __shared__ ull scratch[2 * GC_WAVES_PER_BLOCK];
    const long long na = (long long)c->heavy_cnt, nb = (long long)c->wide_cnt;
    if (na + nb == 0) return;
    const long long kbound = c->kbound;
    const long long maxc = c->maxcolor;
    long long words = (maxc + 2 + 31) / 32;
    words = words < 1 ? 1 : (words > GC_MEX_WORDS ? GC_MEX_WORDS : words);
    long long lmax = -1;
    ull lfail = 0, lsum = 0, lnv = 0;
    // Hubs whose bitmap covers every colour in use: a wave each (first zero bit of a
    // <= 4096-bit bitmap), not a workgroup with its barriers.  Heavy == hub while hubs are on.
    const bool hub_waves = g.hbits_w && maxc + 2 <= 32ll * g.hbits_w;
    if (hub_waves && GC_PB_HUB_LANES) {
        // a run of up to 64 hubs per wave, one per lane: each lane reads its own hub's bitmap
        // words, 8 in flight per step (round 6: a wave per hub walked ~46 hubs of a big round
        // one after another, three dependent trips each)
        const int lane = gc_lane();
        const int w = threadIdx.x / GC_WAVE;
        const long long W = (long long)gridDim.x * GC_WAVES_PER_BLOCK;
        const long long wid = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w;
        const long long per = std::min<long long>(GC_WAVE, std::max<long long>(1, (na + W - 1) / W));
        for (long long i0 = wid * per; i0 < na; i0 += W * per) {
            const long long i = i0 + lane;
            const int v = (lane < per && i < na) ? L.heavy[i] : -1;
            const int x = v >= 0 ? g.hid[v] : -1;
            const int d = v >= 0 ? g.deg[v] : 0;
            long long mex = -1;
            if (x >= 0) {
                for (int t0 = 0; t0 < words && mex < 0; t0 += 8) {
                    unsigned wd[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) wd[k] = t0 + k < words ? *gc_hbw(g, x, t0 + k) : 0xFFFFFFFFu;
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        if (mex < 0 && wd[k] != 0xFFFFFFFFu) mex = 32ll * (t0 + k) + __builtin_ctz(~wd[k]);
                }
                if (g.hub_w) {  // the hub JP's state: this round's conflict flag, cursors, mirror
                    g.hkill[x] = 0u;
                    g.hcur[x] = 0;
                    g.hpc[x] = 0;
                    if (g.hprep) g.hkcnt[x] = 0;
                    g.hk[x] = gc_hk((unsigned)mex, GC_JP_UND);
                }
                gc_set_cand(g, v, mex);
                lmax = mex > lmax ? mex : lmax;
                if (kbound >= 0 && mex >= kbound && (!g.hub_repl || (v >= g.own_lo && v < g.own_hi))) lfail++;
                lsum += (ull)d;
                lnv++;
            }
        }
    } else if (hub_waves) {  // a wave per hub (round 5)
        const int lane = gc_lane();
        const int w = threadIdx.x / GC_WAVE;
        for (long long i = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w; i < na;
             i += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
            const int v = L.heavy[i];
            const int x = g.hid[v];
            long long mex = -1;
            for (int t0 = 0; t0 < words && mex < 0; t0 += GC_WAVE) {  // a zero bit lies in range
                const int t = t0 + lane;
                const unsigned wd = t < words ? *gc_hbw(g, x, t) : 0xFFFFFFFFu;
                const ull m = __ballot(wd != 0xFFFFFFFFu);
                if (m) {
                    const int l = __ffsll((long long)m) - 1;
                    const unsigned zw = __shfl(wd, l, GC_WAVE);
                    mex = 32ll * (t0 + l) + __builtin_ctz(~zw);
                }
            }
            if (lane == 0) {
                if (g.hub_w) {  // the hub JP's state: this round's conflict flag, cursors, mirror
                    g.hkill[x] = 0u;
                    g.hcur[x] = 0;
                    g.hpc[x] = 0;
                    if (g.hprep) g.hkcnt[x] = 0;
                    g.hk[x] = gc_hk((unsigned)mex, GC_JP_UND);
                }
                gc_set_cand(g, v, mex);
                lmax = mex > lmax ? mex : lmax;
                if (kbound >= 0 && mex >= kbound && (!g.hub_repl || (v >= g.own_lo && v < g.own_hi))) lfail++;
                lsum += (ull)g.deg[v];
                lnv++;
            }
        }
    }
    for (long long i = (hub_waves ? na : 0) + blockIdx.x; i < na + nb; i += gridDim.x) {
        const int v = i < na ? L.heavy[i] : L.wide[i - na];
        const int d = g.deg[v];
        const long long start = g.rp[v];
        long long mex = -1;
        const int x = (g.hbits_w && i < na) ? g.hid[v] : -1;
        if (x >= 0) {
            // hub (gc_hubs.hip): forbidden colours pushed by its neighbours' commits; clear
            // its conflict flag for this round
            if (threadIdx.x == 0) {
                if (g.hub_w) {  // the hub JP's state (bitmaps alone: none)
                    g.hkill[x] = 0u;
                    g.hcur[x] = 0;
                    g.hpc[x] = 0;
                    if (g.hprep) g.hkcnt[x] = 0;
                }
                s_first = 0x7FFFFFFF;
            }
            __syncthreads();
            if (maxc + 2 <= 32ll * g.hbits_w) {  // mex <= maxcolor + 1: a zero bit lies in range
                for (int t = threadIdx.x; t < words; t += blockDim.x)
                    if (~*gc_hbw(g, x, t)) atomicMin(&s_first, t);
                __syncthreads();
                mex = 32ll * s_first + __builtin_ctz(~*gc_hbw(g, x, s_first));
            }
            __syncthreads();
        }
        for (long long base = 0; mex < 0; base += 32ll * words) {
            for (int t = threadIdx.x; t < words; t += blockDim.x) s_bits[t] = 0;
            if (threadIdx.x == 0) s_first = 0x7FFFFFFF;
            __syncthreads();
            for (long long e = threadIdx.x; e < d; e += blockDim.x) {
                const long long cc = gc_colour(g, g.col[start + e]) - base;
                if (cc >= 0 && cc < 32ll * words) atomicOr(&s_bits[cc >> 5], 1u << (cc & 31));
            }
            __syncthreads();
            for (int t = threadIdx.x; t < words; t += blockDim.x)
                if (~s_bits[t]) atomicMin(&s_first, t);
            __syncthreads();
            if (s_first != 0x7FFFFFFF) mex = base + 32ll * s_first + __builtin_ctz(~s_bits[s_first]);
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            gc_set_cand(g, v, mex);
            if (x >= 0 && g.hub_w) {  // hub mirror
                g.hk[x] = gc_hk((unsigned)mex, GC_JP_UND);
            }
            lmax = mex > lmax ? mex : lmax;
            if (kbound >= 0 && mex >= kbound && (!g.hub_repl || (v >= g.own_lo && v < g.own_hi))) lfail++;
            lsum += (ull)d;
            lnv++;
        }
    }
    __syncthreads();
    gc_block_max(&c->maxmex, lmax, (long long*)scratch);
    gc_block_add(&c->failcnt, lfail, scratch);
    gc_stat_add(g, GC_K_PROPOSE, lsum, lnv, scratch);
}

// ------------------------------------------------------------------------------------
// resolve (resolve_collisions, coloring.py:56-70) as Jones-Plassmann sweeps.
// v is IN iff every same-candidate listed neighbour u of lower rank is OUT, OUT as soon
// as one is IN.  States only move UND -> IN/OUT, so reading a newer state than the
// sweep started with is harmless (decisions are final).  Every row lists its lower-rank
// neighbours first (nlow[v] of them, fixed at graph creation: rank is static), so a
// sweep walks only those and gathers ONE byte per edge, k8[u] = cand6 << 2 | state;
// cand[] is read only for candidates >= 62.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned gc_jp_flag(const GDev& g, int u, unsigned ku, unsigned cv6, int cv) {
    if (gc_k8_cand(ku) != cv6) return 0u;
    if (cv6 == GC_K8_BIG && g.cand[u] != cv) return 0u;
    const unsigned st = gc_k8_state(ku);
    return st == GC_JP_IN ? 1u : (st == GC_JP_UND ? 2u : 0u);
}

// gc_jp_flag for a hub entry hx (hub index) from the hub mirror hk = gc_hk(candidate, state)
// of the hub, or GC_HK_COLOURED (its candidate field matches no proposal)
__device__ __forceinline__ unsigned gc_jp_flag_h(const GDev& g, int hx, unsigned hk, unsigned cv6, int cv) {
    (void)g; (void)hx; (void)cv6;
    if ((hk >> 2) != (unsigned)cv) return 0u;
    const unsigned st = hk & 3u;
    return st == GC_JP_IN ? 1u : (st == GC_JP_UND ? 2u : 0u);
}

__device__ __forceinline__ void gc_set_state(GDev& g, int v, unsigned kv, unsigned st) {
    g.k8[v] = (unsigned char)((kv & ~3u) | st);
}

// JP step of hub x against the lower-rank hubs of its row (hlow).  The first evaluation
// of a round reads the whole row: undecided entries with the hub's candidate go to its
// pending list, and the entries not yet coloured are copied to the next working copy of
// the row (colours are final, so a coloured entry never matters again: the rows of the
// hubs that linger shrink round by round).  Later sweeps of the round re-check only the
// pending list (ping-pong halves hpend[0|1], hlow's offsets, never overflow).
// hpc[x] = pending count << 1 | current half; hcur[x] = 1 once the row was read this round;
// hrow[x] = which copy holds the live row (0: the original hlow_col), hlen[x] its length.
// Returns 1 (OUT: a same-candidate lower-rank hub is IN), 2 (undecided) or 0 (IN); whole
// workgroup, same value everywhere.
// ... evaluated by ONE wave (all 64 lanes call with the same x; returns the same value on
// every lane).  Hub rows of lower-rank hubs are short (R-MAT-24: at most ~1.7k entries),
// while a hub's evaluation is a chain of ~10 dependent loads: a wave per hub keeps 4x as
// many hubs in flight as a workgroup per hub, and its appends are counted in registers.
// The hub's state words (hpc, hcur, hrow, hlen, hkcnt, hlow_rp) come in prefetched: the
// sweep loads them for 64 hubs at once, one per lane (gc_jp_sweep), instead of as the
// first links of every hub's own chain of dependent loads.
struct GcHubPre {
    long long base, full;  // hlow_rp[x], its static row length
    int enc, hc0, hrow, hlen, hkcnt;
};
__device__ unsigned gc_hub_jp_wave(const GDev& g, int x, unsigned cv6, int cv, GcHubPre p) {
    const int lane = gc_lane();
    const ull lt = gc_lanemask_lt();
    const unsigned* __restrict__ hk = g.hk;  // rows hold hub indices
    int enc = p.enc;
    const int hc0 = p.hc0;
    const bool first = hc0 == 0;
    int hrow = p.hrow, hlen = p.hlen;
    if (hc0 == 2) {  // the grid read this long row in the hub-start sweep (gc_hub_first_long): adopt its
        enc |= 1;    // kept copy and its pending list (half 1)
        hrow = hrow == 1 ? 2 : 1;
        hlen = p.hkcnt;
        if (lane == 0) {
            g.hrow[x] = hrow;
            g.hlen[x] = hlen;
            g.hcur[x] = 1;
        }
    }
    const int sel = enc & 1, cnt = enc >> 1;
    const long long base = p.base;
    const int* __restrict__ src = g.hpend[sel] + base;
    int* dst = g.hpend[sel ^ 1] + base;
    int nn = 0, nk = 0;  // wave-uniform append counts
    bool out = false;    // wave-uniform
    for (int i0 = 0; i0 < cnt && !out; i0 += 4 * GC_WAVE) {  // 4 per lane, flags before stores
        int u[4];
        unsigned fl[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = i0 + k * GC_WAVE + lane;
            u[k] = i < cnt ? src[i] : -1;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) fl[k] = u[k] >= 0 ? (unsigned)hk[u[k]] : 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) fl[k] = u[k] >= 0 ? gc_jp_flag_h(g, u[k], fl[k], cv6, cv) : 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (__ballot((fl[k] & 1u) != 0u)) out = true;
            const ull m = __ballot(fl[k] == 2u);
            if (fl[k] == 2u) dst[nn + __popcll(m & lt)] = u[k];
            nn += __popcll(m);
        }
    }
    const int hr = first ? hrow : 0;
    if (first) {
        const int len = hr ? hlen : (int)p.full;
        const int* __restrict__ hc = g.hlowb[hr] + base;
        int* keep = g.hlowb[hr == 1 ? 2 : 1] + base;
        // GC_HUB_UNR entries per lane in flight; every flag (and its cand[] gather, for
        // candidates >= 62) is computed before the first store, which could alias cand[]
        for (int e0 = 0; e0 < len; e0 += GC_HUB_UNR * GC_WAVE) {
            int u[GC_HUB_UNR];
#pragma unroll
            for (int k = 0; k < GC_HUB_UNR; ++k) {
                const int e = e0 + k * GC_WAVE + lane;
                u[k] = e < len ? hc[e] : -1;
            }
            unsigned ku[GC_HUB_UNR];
#pragma unroll
            for (int k = 0; k < GC_HUB_UNR; ++k) ku[k] = u[k] >= 0 ? (unsigned)hk[u[k]] : GC_HK_COLOURED;
            unsigned fl[GC_HUB_UNR];
#pragma unroll
            for (int k = 0; k < GC_HUB_UNR; ++k) {
                const bool live = ku[k] != GC_HK_COLOURED;  // coloured (or no entry): dropped for good
                fl[k] = live ? 4u | gc_jp_flag_h(g, u[k], ku[k], cv6, cv) : 0u;  // bit 2: live
            }
#pragma unroll
            for (int k = 0; k < GC_HUB_UNR; ++k) {
                if (__ballot((fl[k] & 1u) != 0u)) out = true;
                const ull mk = __ballot(fl[k] != 0u);
                if (fl[k]) keep[nk + __popcll(mk & lt)] = u[k];
                nk += __popcll(mk);
                const ull mp = __ballot((fl[k] & 3u) == 2u);
                if ((fl[k] & 3u) == 2u) dst[nn + __popcll(mp & lt)] = u[k];
                nn += __popcll(mp);
            }
        }
    }
    if (lane == 0) {
        if (first) {  // the kept copy is complete (the whole row was read)
            g.hrow[x] = hr == 1 ? 2 : 1;
            g.hlen[x] = nk;
            g.hcur[x] = 1;
        }
        if (!out) g.hpc[x] = (nn << 1) | (sel ^ 1);
    }
    return out ? 1u : (nn > 0 ? 2u : 0u);
}

// JP step of hub x by a resumable scan of its row (hubs on, GC_HUB_SCAN; the default).
// Hub indices are assigned in rank order (gc_hubs.hip) and every hlow row is sorted by
// them, so the row lists the hub's lower-rank hubs lowest rank first.  The hub walks it
// from where it stopped: an entry coloured, OUT or of another candidate can never block
// it again this round (states only move UND -> IN / OUT inside a round, candidates are
// fixed), so the walk stops at the first same-candidate UNDECIDED entry (the cursor, hpc),
// and the hub is OUT as soon as a same-candidate entry is IN, IN once the end is reached.
// Exactly the JP rule over the row, with no per-round copies: the kept-row and
// pending-list rewrites of gc_hub_jp_wave wrote ~2x the live rows every round (R-MAT-24:
// 60 GB of writes per colouring in the sweeps), and lower-rank winners sit near the row
// start, so an OUT hub usually stops early.  Colours are final, so the coloured prefix of
// the row is skipped for good: hlen holds its length (reset per colouring).
// p.hc0 = hcur (0: first evaluation this round), p.enc = cursor, p.hlen = coloured prefix.
__device__ unsigned gc_hub_scan_wave(const GDev& g, int x, unsigned cv6, int cv, GcHubPre p) {
    const int lane = gc_lane();
    const unsigned* __restrict__ hk = g.hk;  // rows hold hub indices
    const bool first = p.hc0 == 0;
    const int full = (int)p.full;
    const int* __restrict__ row = g.hlow_col + p.base;
    int pos = first ? p.hlen : p.enc;
    bool out = false, prefix = first;
    int block = -1, nstart = full;
    for (int e0 = pos; e0 < full && !out && block < 0; e0 += GC_HUB_UNR * GC_WAVE) {
        int u[GC_HUB_UNR];
#pragma unroll
        for (int k = 0; k < GC_HUB_UNR; ++k) {
            const int e = e0 + k * GC_WAVE + lane;
            u[k] = e < full ? row[e] : -1;
        }
        unsigned ku[GC_HUB_UNR];
#pragma unroll
        for (int k = 0; k < GC_HUB_UNR; ++k) ku[k] = u[k] >= 0 ? (unsigned)hk[u[k]] : GC_HK_COLOURED;
        unsigned fl[GC_HUB_UNR];
#pragma unroll
        for (int k = 0; k < GC_HUB_UNR; ++k) fl[k] = ku[k] != GC_HK_COLOURED ? gc_jp_flag_h(g, u[k], ku[k], cv6, cv) : 0u;
#pragma unroll
        for (int k = 0; k < GC_HUB_UNR; ++k) {
            if (__ballot(fl[k] == 1u)) out = true;
            const ull mb = __ballot(fl[k] == 2u);
            if (mb && block < 0) block = e0 + k * GC_WAVE + __builtin_ctzll(mb);
            if (prefix) {  // first non-coloured entry: the end of the coloured prefix
                const ull ml = __ballot(u[k] >= 0 && ku[k] != GC_HK_COLOURED);
                if (ml) {
                    nstart = e0 + k * GC_WAVE + __builtin_ctzll(ml);
                    prefix = false;
                }
            }
        }
    }
    if (lane == 0) {
        if (first) {
            g.hcur[x] = 1;
            if (nstart > p.hlen) g.hlen[x] = nstart;
        }
        if (!out && block >= 0) g.hpc[x] = block;
    }
    return out ? 1u : (block >= 0 ? 2u : 0u);
}

// The resumable scan (gc_hub_scan_wave) of GC_HUB_NG hubs at once, one group of
// GC_WAVE / GC_HUB_NG lanes each: a hub's scan usually ends in its first step (at its first
// same-candidate undecided entry, or at an IN one), so a wave that walked its hubs one after
// another paid a chain of dependent loads per hub -- the hub-start sweep's floor.  The
// hubs' state comes prefetched, one per lane (slot j of the prefetch = lane j).
#ifndef GC_HUB_NG
#define GC_HUB_NG 8  // (4: R-MAT-26 +1.0%, R-MAT-24 +-0.5%; 16: R-MAT-24 +4%, profiles/r06/n)
#endif
__device__ void gc_hub_scan_groups(GDev& g, int nj, int pv, unsigned pkv, int pcv, int px, unsigned pkill,
                                   const GcHubPre& pp, GcStage& st, int* ho, ull* ho_cnt, ull& lsum, ull& lnv,
                                   long long* dout, ull* dcnt) {
    constexpr int GS = GC_WAVE / GC_HUB_NG;
    const int lane = gc_lane();
    const int grp = lane / GS, li = lane % GS;
    const ull gmask = ((1ull << GS) - 1ull) << (grp * GS);
    const unsigned* __restrict__ hk = g.hk;
    for (int j0 = 0; j0 < nj; j0 += GC_HUB_NG) {
        const int j = j0 + grp;
        const bool has = j < nj;
        const int jj = has ? j : 0;
        const int v = __shfl(pv, jj, GC_WAVE);
        const unsigned kv = (unsigned)__shfl((int)pkv, jj, GC_WAVE);
        const unsigned cv6 = gc_k8_cand(kv);
        const int cv = __shfl(pcv, jj, GC_WAVE);
        const int xs = __shfl(px, jj, GC_WAVE);  // every lane takes part in every shuffle: a
        const int x = has ? xs : -1;              // disabled source lane would read back 0
        const bool kill = __shfl((int)pkill, jj, GC_WAVE) != 0;
        const long long base = __shfl(pp.base, jj, GC_WAVE);
        const int full = (int)__shfl(pp.full, jj, GC_WAVE);
        const int cursor = __shfl(pp.enc, jj, GC_WAVE);
        const int hc0 = __shfl(pp.hc0, jj, GC_WAVE);
        const int hstart = __shfl(pp.hlen, jj, GC_WAVE);
        const bool act = has && x >= 0 && !kill;  // group-uniform
        const bool first = hc0 == 0;
        int pos = first ? hstart : cursor;
        bool out = false, prefix = act && first;
        int block = -1, nstart = full;
        const int* __restrict__ row = g.hlow_col + base;
        for (;;) {
            const bool run = act && !out && block < 0 && pos < full;
            if (!__ballot(run)) break;
            int u[GC_HUB_UNR];
#pragma unroll
            for (int k = 0; k < GC_HUB_UNR; ++k) {
                const int e = pos + k * GS + li;
                u[k] = (run && e < full) ? row[e] : -1;
            }
            unsigned ku[GC_HUB_UNR];
#pragma unroll
            for (int k = 0; k < GC_HUB_UNR; ++k) ku[k] = u[k] >= 0 ? (unsigned)hk[u[k]] : GC_HK_COLOURED;
            unsigned fl[GC_HUB_UNR];
#pragma unroll
            for (int k = 0; k < GC_HUB_UNR; ++k) fl[k] = ku[k] != GC_HK_COLOURED ? gc_jp_flag_h(g, u[k], ku[k], cv6, cv) : 0u;
#pragma unroll
            for (int k = 0; k < GC_HUB_UNR; ++k) {
                if (__ballot(fl[k] == 1u) & gmask) out = true;
                const ull mb = __ballot(fl[k] == 2u) & gmask;
                if (mb && block < 0) block = pos + k * GS + __builtin_ctzll(mb >> (grp * GS));
                const ull ml = __ballot(u[k] >= 0 && ku[k] != GC_HK_COLOURED) & gmask;
                if (prefix && ml) {  // first non-coloured entry: the end of the coloured prefix
                    nstart = pos + k * GS + __builtin_ctzll(ml >> (grp * GS));
                    prefix = false;
                }
            }
            if (run) pos += GC_HUB_UNR * GS;
        }
        unsigned f = kill ? 1u : 0u;
        const bool lead = li == 0 && has && x >= 0;
        if (act) {
            f = out ? 1u : (block >= 0 ? 2u : 0u);
            if (li == 0) {
                if (first) {
                    g.hcur[x] = 1;
                    if (nstart > hstart) g.hlen[x] = nstart;
                }
                if (!out && block >= 0) g.hpc[x] = block;
            }
        }
        gc_stage_push(st, lead && (f & 3u) == 2u, v, ho, ho_cnt);  // undecided hub
        if (lead) {
            if (f & 1u) gc_set_state(g, v, kv, GC_JP_OUT);
            else if (!(f & 2u)) gc_set_state(g, v, kv, GC_JP_IN);
            if ((f & 1u) || !(f & 2u))  // hub mirror
                g.hk[x] = gc_hk((unsigned)cv, (f & 1u) ? GC_JP_OUT : GC_JP_IN);
            if (dout && ((f & 1u) || !(f & 2u)))
                dout[atomicAdd(dcnt, 1ull)] = gc_delta(v, (f & 1u) ? GC_JP_OUT : GC_JP_IN);
            lsum += (ull)g.deg[v];
            lnv++;
        }
        // not a hub (cannot happen while heavy_t is the hub threshold): row scan, a wave each
        ull nh = __ballot(li == 0 && has && x < 0);
        while (nh) {
            const int l = __ffsll((long long)nh) - 1;
            nh &= nh - 1;
            const int vv = __shfl(v, l, GC_WAVE);
            const unsigned kvv = (unsigned)__shfl((int)kv, l, GC_WAVE);
            const unsigned c6 = gc_k8_cand(kvv);
            const int cvv = __shfl(cv, l, GC_WAVE);
            const int dl = g.nlow[vv];
            const long long start = g.rp[vv];
            unsigned lf = 0;
            for (int e = lane; e < dl; e += GC_WAVE) {
                const int uu = g.col[start + e];
                lf |= gc_jp_flag(g, uu, g.k8[uu], c6, cvv);
            }
            const unsigned ff = (__ballot((lf & 1u) != 0u) ? 1u : 0u) | (__ballot((lf & 2u) != 0u) ? 2u : 0u);
            gc_stage_push(st, lane == 0 && (ff & 3u) == 2u, vv, ho, ho_cnt);
            if (lane == 0) {
                if (ff & 1u) gc_set_state(g, vv, kvv, GC_JP_OUT);
                else if (!(ff & 2u)) gc_set_state(g, vv, kvv, GC_JP_IN);
                if (dout && ((ff & 1u) || !(ff & 2u)))
                    dout[atomicAdd(dcnt, 1ull)] = gc_delta(vv, (ff & 1u) ? GC_JP_OUT : GC_JP_IN);
                lsum += (ull)g.deg[vv];
                lnv++;
            }
        }
    }
}

// First read of the LONG hub rows (static length > hub_long) in the sweep that starts the
// hubs, by the whole grid: one wave per GC_HCH-entry chunk (static chunk index hch_rp /
// hch_own, scanned in a scattered order so a long row's chunks land on many waves).  It
// writes what the hub's first evaluation would: the kept copy of the row (uncoloured
// entries; hkcnt counts them) and the pending list (entries with the hub's candidate that
// are not OUT, in hpend[1]; hpc counts them, x2).  The hub itself was listed undecided with
// hcur = 2 by the same sweep and adopts both at its first evaluation (next sweep).  No hub
// is IN before this sweep's evaluations; an entry that is IN by the time the hub reads its
// pending list makes it OUT there, as in the row walk.  One wave walking a 2.5e5-entry row
// (R-MAT-26) was the hub-start sweep's long pole.
__device__ void gc_hub_first_long(GDev& g) {
    constexpr int K = GC_HCH / GC_WAVE;
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    const ull lt = gc_lanemask_lt();
    const unsigned* __restrict__ hk = g.hk;  // rows hold hub indices
    const long long NC = g.nhch;
    const long long wstride = (long long)gridDim.x * GC_WAVES_PER_BLOCK * GC_WAVE;
    for (long long j0 = ((long long)blockIdx.x * GC_WAVES_PER_BLOCK + w) * GC_WAVE; j0 < NC; j0 += wstride) {
        const long long j = j0 + lane;
        int x = -1, part = 0, len = 0, hr = 0;
        unsigned kx = 0;
        if (j < NC) {
            const long long jj = (long long)(((ull)j * (ull)g.hch_mul) % (ull)NC);
            x = g.hch_own[jj];
            part = (int)(jj - g.hch_rp[x]);
            const long long full = g.hlow_rp[x + 1] - g.hlow_rp[x];
            if (full > g.hub_long) {
                kx = hk[x];
                hr = g.hrow[x];
                len = hr ? g.hlen[x] : (int)full;
            }
            // short row / no proposer / past the live row / flagged (OUT without a read)
            if (full <= g.hub_long || kx == GC_HK_COLOURED || (kx >> 2) == GC_HK_NOCAND || (long long)part * GC_HCH >= len ||
                g.hkill[x])
                x = -1;
        }
        ull act = __ballot(x >= 0);
        while (act) {
            const int sl = __ffsll((long long)act) - 1;
            act &= act - 1;
            const int hx = __shfl(x, sl, GC_WAVE);
            const int e0 = __shfl(part, sl, GC_WAVE) * GC_HCH;
            const int hl = __shfl(len, sl, GC_WAVE);
            const int hhr = __shfl(hr, sl, GC_WAVE);
            const int cv = (int)(__shfl(kx, sl, GC_WAVE) >> 2);
            const unsigned cv6 = gc_c6_of(cv);
            const long long base = g.hlow_rp[hx];
            const int* __restrict__ hc = g.hlowb[hhr] + base;
            int u[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int e = e0 + k * GC_WAVE + lane;
                u[k] = e < hl ? hc[e] : -1;
            }
            unsigned ku[K];
#pragma unroll
            for (int k = 0; k < K; ++k) ku[k] = u[k] >= 0 ? (unsigned)hk[u[k]] : GC_HK_COLOURED;
            ull mk[K], mp[K];  // wave masks per slot: live (kept) / pending
            int tk = 0, tp = 0;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const bool live = ku[k] != GC_HK_COLOURED;  // coloured (or no entry): dropped for good
                mk[k] = __ballot(live);
                mp[k] = __ballot(live && gc_jp_flag_h(g, u[k], ku[k], cv6, cv) != 0u);
                tk += __popcll(mk[k]);
                tp += __popcll(mp[k]);
            }
            int kb = 0, pb = 0;
            if (lane == 0) {
                if (tk) kb = atomicAdd(&g.hkcnt[hx], tk);
                if (tp) pb = atomicAdd(&g.hpc[hx], 2 * tp) >> 1;
            }
            kb = __shfl(kb, 0, GC_WAVE);
            pb = __shfl(pb, 0, GC_WAVE);
            int* keep = g.hlowb[hhr == 1 ? 2 : 1] + base;
            int* pend = g.hpend[1] + base;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if ((mk[k] >> lane) & 1ull) keep[kb + __popcll(mk[k] & lt)] = u[k];
                if ((mp[k] >> lane) & 1ull) pend[pb + __popcll(mp[k] & lt)] = u[k];
                kb += __popcll(mk[k]);
                pb += __popcll(mp[k]);
            }
        }
    }
}

// One JP sweep over a light list (wave chunks) and a heavy list (workgroup per vertex);
// undecided vertices are appended to (uo, uo_cnt) / (ho, ho_cnt).
template <int NW = GC_WAVES_PER_BLOCK>
__device__ __forceinline__ void gc_jp_sweep(GDev& g, const int* __restrict__ list, long long cnt, int skip_heavy,
                                            const int* hlist, long long hcnt, int* uo, ull* uo_cnt, int* ho,
                                            ull* ho_cnt, ull& lsum, ull& lnv, long long* dout, ull* dcnt,
                                            bool hub_first = false) {
    __shared__ unsigned s_flag[NW][GC_WAVE];
    __shared__ int s_first[NW][GC_WAVE];
    __shared__ long long s_start[NW][GC_WAVE];
    __shared__ unsigned s_c6[NW][GC_WAVE];
    __shared__ int s_cv[NW][GC_WAVE];
    __shared__ unsigned s_f;
    __shared__ int s_stage[NW][GC_STAGE_CAP];
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    const unsigned char* __restrict__ k8 = g.k8;
    // undecided appends staged in LDS: one atomic per 512 entries, not one per wave-chunk
    // (a single counter takes ~88 returning atomics/us; 86k chunks cost ~1 ms)
    GcStage st{s_stage[w], 0, g.list_cap, &g.ctl->loop_err, &g.ctl->halt};
    // heavy vertices first.  Hubs off: a workgroup each, undecided ones staged by wave 0
    __shared__ int s_hstage[GC_STAGE_CAP];
    GcStage hst{s_hstage, 0, g.list_cap, &g.ctl->loop_err, &g.ctl->halt};
    long long* const hdout = g.hub_repl ? nullptr : dout;  // replicated hubs (shards) are never sent
    if (g.hub_w) {  // hubs on: a wave per hub (gc_hub_jp_wave), undecided staged per wave
        // a wave's hubs are i = wid + j * waves; lane l loads the state of hub j0 + l, so a
        // hub's evaluation starts at its row read
        const long long waves = (long long)gridDim.x * NW;
        const long long wid = (long long)blockIdx.x * NW + w;
        for (long long i0 = wid; i0 < hcnt; i0 += waves * GC_WAVE) {
            const long long il = i0 + (long long)lane * waves;
            int pv = -1, px = -1, pcv = 0;
            unsigned pkv = 0, pkill = 0;
            GcHubPre pp{0, 0, 0, 0, 0, 0, 0};
            if (il < hcnt) {
                pv = hlist[il];
                pkv = k8[pv];
                pcv = gc_k8_cand(pkv) == GC_K8_BIG ? g.cand[pv] : (int)gc_k8_cand(pkv);
                px = g.hid[pv];
            }
            if (px >= 0) {
                pkill = g.hkill[px];
                pp.base = g.hlow_rp[px];
                pp.full = g.hlow_rp[px + 1] - pp.base;
                pp.enc = g.hpc[px];
                pp.hc0 = g.hcur[px];
                pp.hrow = g.hrow[px];
                pp.hlen = g.hlen[px];
                pp.hkcnt = g.hkcnt[px];
            }
            const long long left = (hcnt - i0 + waves - 1) / waves;
            const int nj = left < GC_WAVE ? (int)left : GC_WAVE;
            if (g.hub_scan) {
                gc_hub_scan_groups(g, nj, pv, pkv, pcv, px, pkill, pp, st, ho, ho_cnt, lsum, lnv, hdout, dcnt);
                continue;
            }
            for (int j = 0; j < nj; ++j) {
                const int v = __shfl(pv, j, GC_WAVE);
                const unsigned kv = (unsigned)__shfl((int)pkv, j, GC_WAVE);
                const unsigned cv6 = gc_k8_cand(kv);
                const int cv = __shfl(pcv, j, GC_WAVE);
                const int x = __shfl(px, j, GC_WAVE);
                unsigned f = 0;
                if (x >= 0) {
                    GcHubPre q;
                    q.base = __shfl(pp.base, j, GC_WAVE);
                    q.full = __shfl(pp.full, j, GC_WAVE);
                    q.enc = __shfl(pp.enc, j, GC_WAVE);
                    q.hc0 = __shfl(pp.hc0, j, GC_WAVE);
                    q.hrow = __shfl(pp.hrow, j, GC_WAVE);
                    q.hlen = __shfl(pp.hlen, j, GC_WAVE);
                    q.hkcnt = __shfl(pp.hkcnt, j, GC_WAVE);
                    if (__shfl((int)pkill, j, GC_WAVE)) {
                        f = 1u;
                    } else if (g.hub_scan) {
                        f = gc_hub_scan_wave(g, x, cv6, cv, q);
                    } else if (hub_first && q.full > g.hub_long) {
                        f = 2u;  // long row: read by the grid below (gc_hub_first_long), evaluated next sweep
                        if (lane == 0) g.hcur[x] = 2;
                    } else {
                        f = gc_hub_jp_wave(g, x, cv6, cv, q);
                    }
                } else {  // not a hub (cannot happen while heavy_t is the hub threshold): row scan
                    const int dl = g.nlow[v];
                    const long long start = g.rp[v];
                    unsigned lf = 0;
                    for (int e = lane; e < dl; e += GC_WAVE) {
                        const int u = g.col[start + e];
                        lf |= gc_jp_flag(g, u, k8[u], cv6, cv);
                    }
                    f = (__ballot((lf & 1u) != 0u) ? 1u : 0u) | (__ballot((lf & 2u) != 0u) ? 2u : 0u);
                }
                gc_stage_push(st, lane == 0 && (f & 3u) == 2u, v, ho, ho_cnt);  // undecided hub
                if (lane == 0) {
                    if (f & 1u) gc_set_state(g, v, kv, GC_JP_OUT);
                    else if (!(f & 2u)) gc_set_state(g, v, kv, GC_JP_IN);
                    if (x >= 0 && ((f & 1u) || !(f & 2u)))  // hub mirror
                        g.hk[x] = gc_hk((unsigned)cv, (f & 1u) ? GC_JP_OUT : GC_JP_IN);
                    if (hdout && ((f & 1u) || !(f & 2u)))
                        hdout[atomicAdd(dcnt, 1ull)] = gc_delta(v, (f & 1u) ? GC_JP_OUT : GC_JP_IN);
                    lsum += (ull)g.deg[v];
                    lnv++;
                }
            }
        }
        gc_stage_flush(st, ho, ho_cnt);  // st is the light list's stage from here on
        if (hub_first && !g.hub_scan) gc_hub_first_long(g);
        hcnt = 0;
    }
    // Hubs off here (hubs on: evaluated by waves above, hcnt = 0).  The round's first sweep
    // scans v's lower-rank part and keeps the entries that can still block v (same
    // candidate, undecided) in v's pending list (g.hpl at rp[v], when allocated); later
    // sweeps read only that list, compacting it in place (a survivor's new slot never
    // passes an entry not yet read).  A same-candidate IN entry ends the scan: v is OUT.
    // Hubs-off R-MAT-24 (the shards' engine): 2.44 -> 1.62 s.
    __shared__ int s_pc;
    for (long long i = blockIdx.x; i < hcnt; i += gridDim.x) {
        const int v = hlist[i];
        const int d = g.deg[v];
        const long long start = g.rp[v];
        const unsigned kv = k8[v];
        const unsigned cv6 = gc_k8_cand(kv);
        const int cv = cv6 == GC_K8_BIG ? g.cand[v] : (int)cv6;
        int* pl = g.hpl ? g.hpl + start : nullptr;
        const bool fresh = skip_heavy || !pl;  // resolve: the round's first sweep
        const int len = fresh ? g.nlow[v] : g.hplc[v];
        const int* src = fresh ? g.col + start : pl;
        if (threadIdx.x == 0) {
            s_f = 0;
            s_pc = 0;
        }
        __syncthreads();
        for (int e0 = 0; e0 < len; e0 += blockDim.x) {
            const int e = e0 + (int)threadIdx.x;
            int u = 0;
            unsigned f = 0;
            if (e < len) {
                u = src[e];
                f = gc_jp_flag(g, u, k8[u], cv6, cv);
            }
            if (f) atomicOr(&s_f, f);
            __syncthreads();  // the chunk is read before any survivor is written back
            if (pl && f == 2u) pl[atomicAdd(&s_pc, 1)] = u;
            __syncthreads();
            const bool out = (s_f & 1u) != 0u;
            __syncthreads();
            if (out) break;
        }
        const unsigned ff = (s_f & 1u) ? 1u : (s_f & 2u);
        if (pl && threadIdx.x == 0) g.hplc[v] = s_pc;
        if (w == 0) gc_stage_push(hst, lane == 0 && (ff & 3u) == 2u, v, ho, ho_cnt);  // undecided hub
        if (threadIdx.x == 0) {
            if (ff & 1u) gc_set_state(g, v, kv, GC_JP_OUT);
            else if (!(ff & 2u)) gc_set_state(g, v, kv, GC_JP_IN);
            if (dout && ((ff & 1u) || !(ff & 2u)))
                dout[atomicAdd(dcnt, 1ull)] = gc_delta(v, (ff & 1u) ? GC_JP_OUT : GC_JP_IN);
            lsum += (ull)d;
            lnv++;
        }
        __syncthreads();
    }
    if (w == 0) gc_stage_flush(hst, ho, ho_cnt);
    const int vpw = gc_vpw(cnt, (long long)gridDim.x * NW);
    const long long nch = gc_nchunks(cnt, vpw);
    for (long long ch = (long long)blockIdx.x * NW + w; ch < nch;
         ch += (long long)gridDim.x * NW) {
        const long long idx = ch * vpw + lane;
        const int v = (lane < vpw && idx < cnt) ? list[idx] : -1;
        // the vertex's words are loaded together (none waits on another: one memory trip)
        const int d = v >= 0 ? g.deg[v] : 0;
        const int lc0 = (v >= 0 && !skip_heavy) ? g.lcur[v] : 0;
        const int nl0 = v >= 0 ? g.nlow[v] : 0;
        const unsigned kv0 = v >= 0 ? (unsigned)k8[v] : 0xFFu;
        const long long rs0 = v >= 0 ? g.rp[v] : 0;
#if GC_HOIST_HIN
        // with the vertex's other words (one trip): its candidate past 61 and its hub-list
        // bounds, so neither is a dependent trip of its own later (round 6)
        const int cb0 = v >= 0 ? g.cand[v] : 0;
        const long long hs0 = (v >= 0 && g.hub_w) ? g.hin_rp[v] : 0;
        const long long he0 = (v >= 0 && g.hub_w) ? g.hin_rp[v + 1] : 0;
#endif
        const bool skip = v < 0 || (skip_heavy && d > g.heavy_t);
        // resumable: entries before lcur[v] were seen decided-not-IN or off-candidate in an
        // earlier sweep of this round (states only move UND -> IN/OUT), so skip them
        const int lc = skip ? 0 : lc0;
        const int dl = skip ? 0 : nl0 - lc;
        const unsigned kv = skip ? 0xFFu : kv0;
        const unsigned cv6 = skip ? 0x100u : gc_k8_cand(kv);
        s_flag[w][lane] = 0;
        s_first[w][lane] = 0x7FFFFFFF;
        s_start[w][lane] = v >= 0 ? rs0 + lc : 0;
        s_c6[w][lane] = cv6;
#if GC_HOIST_HIN
        s_cv[w][lane] = cv6 == GC_K8_BIG ? cb0 : (int)cv6;
#else
        s_cv[w][lane] = cv6 == GC_K8_BIG ? g.cand[v] : (int)cv6;
#endif
        const int incl = gc_wave_incl_scan(dl);
        const int excl = incl - dl;
        const int total = __shfl(incl, GC_WAVE - 1, GC_WAVE);
        gc_wave_sync();
        gc_chunk_edges_at(
            g.col, s_start[w], excl, total, [&](int u) { return (unsigned)k8[u]; },
            [&](int o, int u, unsigned ku, int slot) {
                const unsigned f = gc_jp_flag(g, u, ku, s_c6[w][o], s_cv[w][o]);
                if (f) atomicOr(&s_flag[w][o], f);
                if (f == 2u) atomicMin(&s_first[w][o], slot);
            });
        gc_wave_sync();
        bool pend = false;
        unsigned nst = GC_JP_UND;
        if (!skip) {
            const unsigned f = s_flag[w][lane];
            if (f & 1u) nst = GC_JP_OUT;
            else if (f & 2u) pend = true;
            else nst = GC_JP_IN;
            if (pend) g.lcur[v] = lc + s_first[w][lane];
            if (nst != GC_JP_UND) gc_set_state(g, v, kv, nst);
            lsum += (ull)d;
            lnv++;
        }
        if (dout) gc_wave_append64(nst != GC_JP_UND, gc_delta(v, (int)nst), dout, dcnt);
        gc_stage_push(st, pend, v, uo, uo_cnt);
        if (g.hub_w) {  // a light winner flags the hubs listing it that propose its colour
            int dh = 0;
            long long hs = 0;
            if (nst == GC_JP_IN) {
#if GC_HOIST_HIN
                hs = hs0;
                dh = (int)(he0 - hs0);
#else
                hs = g.hin_rp[v];
                dh = (int)(g.hin_rp[v + 1] - hs);
#endif
            }
            gc_wave_sync();
            s_start[w][lane] = hs;
            const int hincl = gc_wave_incl_scan(dh);
            const int hexcl = hincl - dh;
            const int htotal = __shfl(hincl, GC_WAVE - 1, GC_WAVE);
            gc_wave_sync();
            gc_chunk_edges(
                g.hin_col, s_start[w], hexcl, htotal, [&](int hx) { return g.hk[hx]; },
                [&](int o, int hx, unsigned kh) {  // the hub proposes the winner's colour
                    if ((kh >> 2) != (unsigned)s_cv[w][o]) return;
                    if (!g.hkill[hx]) g.hkill[hx] = 1u;
                });
        }
    }
#ifndef GC_WAVE_FLUSH_MAX
#define GC_WAVE_FLUSH_MAX 0
#endif
    if (cnt <= GC_WAVE_FLUSH_MAX) gc_stage_flush(st, uo, uo_cnt);  // short lists: few waves append, no barriers
    else gc_stage_flush_block<NW>(st, uo, uo_cnt);
}

__global__ void __launch_bounds__(GC_BLOCK) k_resolve(GDev g, GLists L) {
    DevCtl* c = g.ctl;
    if (c->halt) return;
    __shared__ ull scratch[2 * GC_WAVES_PER_BLOCK];
    if (c->kbound >= 0 && c->failcnt > 0) {  // coloring.py:104-108: fail with the round-start state
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            const long long r = c->round;
            RoundRec* rec = L.rec + (r - c->rbase);
            rec->U = c->U;
            rec->F = (long long)c->fcnt[c->cur];
            rec->maxmex = c->maxmex;
            rec->accepted = 0;
            rec->seeds = 0;
            rec->sweeps = 0;
            c->fail_round = r;
            c->fail_count = (long long)c->failcnt;
            c->round = r + 1;
            c->halt = GC_H_FAILED;
        }
        return;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        c->und_cnt[1] = 0;
        c->undh_cnt[1] = 0;
        c->sweeps = 1;
    }
    const int cur = c->cur;
    ull lsum = 0, lnv = 0;
    // hubs sit out the sweeps until the lights have converged (gc_hubs.hip)
    gc_jp_sweep(g, L.F[cur], (long long)c->fcnt[cur], 1, L.heavy, g.hub_w ? 0ll : (long long)c->heavy_cnt, L.undL[0],
                &c->und_cnt[0], L.undH[0], &c->undh_cnt[0], lsum, lnv, L.delta, &c->dcnt);
    __syncthreads();
    gc_stat_add(g, GC_K_RESOLVE, lsum, lnv, scratch);
}

// Sweep i >= 1 reads slot (i-1)%3, appends to slot i%3 and clears slot (i+1)%3, which
// sweep i+1 appends to (its previous reader, sweep i-1, has finished).
__global__ void __launch_bounds__(GC_BLOCK) k_sweep(GDev g, GLists L, int i) {
    DevCtl* c = g.ctl;
    if (c->halt) return;
#if GC_SWEEP_STATS
    __shared__ ull scratch[2 * GC_WAVES_PER_BLOCK];
#endif
    const int in = (i - 1) % 3, out = i % 3, z = (i + 1) % 3;
    const long long cl = (long long)c->und_cnt[in];
    long long ch = (long long)c->undh_cnt[in];
    const int* hl = L.undH[in];
    const bool hub_start = gc_hub_gate(g, c, i, cl, hl, ch, L);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        c->und_cnt[z] = 0;
        c->undh_cnt[z] = 0;
        if (cl + ch > 0) c->sweeps += 1;
        if (cl > g.tail_lmax || ch > gc_tail_hmax(g)) c->bigsweeps = i;
        if (cl > GC_LOOP_MAX || ch > GC_LOOP_HMAX) c->hugesweeps = i;
        if (hub_start) c->hub_start = i;
    }
    if (cl + ch == 0) return;
    ull lsum = 0, lnv = 0;
    gc_jp_sweep(g, L.undL[in], cl, 0, hl, ch, L.undL[out], &c->und_cnt[out], L.undH[out],
                &c->undh_cnt[out], lsum, lnv, L.delta, &c->dcnt, hub_start && g.hprep);
#if GC_SWEEP_STATS  // the sweeps carry no §8d credit (their counts are only diagnostics)
    __syncthreads();
    gc_stat_add(g, GC_K_SWEEP, lsum, lnv, scratch);
#endif
}

// Grid barrier of k_sweep_loop (cdna_hip_programming.md §6 G16): every wave drains its
// stores, the workgroup meets, lane 0 writes back its XCD's L2 (agent release), arrives on
// the monotonic counter and polls it (relaxed, s_sleep), then invalidates its CU's L1
// (agent acquire) before the workgroup reads what the other workgroups wrote.  The wait is
// bounded: a give-up sets DevCtl.loop_err (the host turns it into an error).
__device__ __forceinline__ void gc_grid_barrier(DevCtl* c, unsigned& target, int* s_err) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        target += gridDim.x;
        __hip_atomic_fetch_add(&c->bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        int err = 0;
        while (__hip_atomic_load(&c->bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1u << 24)) {  // far beyond any real wait: give up instead of hanging
                err = 1;
                __hip_atomic_store(&c->loop_err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        *s_err = err | __hip_atomic_load(&c->loop_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
}

// The middle of a round's JP chain in ONE launch: after the host's full-grid sweeps (lists
// past the loop limits), every later sweep whose lists still exceed the one-workgroup tail's
// limits runs here, a grid barrier apart, on a grid every workgroup of which is resident
// (one per CU).  Each such sweep used to be a full-grid launch of ~8-50 us: on R-MAT-26
// ~12 launches a round, 60% of the sweeps' time.  Sweep bookkeeping as k_sweep.
__global__ void __launch_bounds__(GC_BLOCK) k_sweep_loop(GDev g, GLists L, int S) {
    DevCtl* c = g.ctl;
    if (c->halt) return;
    __shared__ ull scratch[2 * GC_WAVES_PER_BLOCK];
    __shared__ long long s_cl, s_ch;
    __shared__ int s_err;
    unsigned target = c->bar_base;
    int j = S;
    ull lsum = 0, lnv = 0;
    for (;;) {
        const int in = j % 3;
        if (threadIdx.x == 0) {
            s_cl = (long long)__hip_atomic_load(&c->und_cnt[in], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_ch = (long long)__hip_atomic_load(&c->undh_cnt[in], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        const long long cl = s_cl;
        long long ch = s_ch;
        const int* hl = L.undH[in];
        const bool hub_start = gc_hub_gate(g, c, j + 1, cl, hl, ch, L);
        // empty, or small enough for the one-workgroup tail (k_sweep_tail takes it from here)
        if (cl + ch == 0 || (cl <= g.tail_lmax && ch <= gc_tail_hmax(g))) break;
        ++j;
        const int out = j % 3, z = (j + 1) % 3;
        __syncthreads();  // every workgroup has read hub_start before block 0 moves it
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            c->und_cnt[z] = 0;
            c->undh_cnt[z] = 0;
            c->sweeps += 1;
            c->bigsweeps = j;
            if (cl > GC_LOOP_MAX || ch > GC_LOOP_HMAX) c->hugesweeps = j;
            if (hub_start) c->hub_start = j;
        }
        gc_jp_sweep(g, L.undL[in], cl, 0, hl, ch, L.undL[out], &c->und_cnt[out], L.undH[out], &c->undh_cnt[out], lsum,
                    lnv, L.delta, &c->dcnt, hub_start && g.hprep);
        gc_grid_barrier(c, target, &s_err);
        if (s_err) break;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        c->loop_last = j;
        c->bar_base = target;
    }
    gc_stat_add(g, GC_K_SWEEP, lsum, lnv, scratch);
}

// The rest of a round's sweeps in ONE workgroup, after the host's S full-grid sweeps: the
// deep end of a JP resolution is a chain of sweeps over a few hundred vertices each, which
// as separate 2048-workgroup launches cost a launch gap apiece (and the sweeps enqueued
// beyond the round's depth ran idle).  Here they run back to back, a workgroup barrier
// apart, while the undecided lists stay within tail_lmax / tail_hmax; a bigger list
// is left to full-grid sweeps (the commit then asks the host for them, GC_H_SWEEPS).
// Counters are read with atomic RMWs and cleared with agent-scope stores; list entries and
// states written before a barrier are visible to the whole workgroup after it.
template <int NW>
__global__ void __launch_bounds__(NW * GC_WAVE) k_sweep_tail(GDev g, GLists L, int S) {
    DevCtl* c = g.ctl;
    if (c->halt) return;
#if GC_SWEEP_STATS
    __shared__ ull scratch[2 * NW];
#endif
    __shared__ long long s_cl, s_ch;
    int j = c->loop_last > S ? (int)c->loop_last : S;  // after k_sweep_loop's sweeps, if it ran
    ull lsum = 0, lnv = 0;
    for (;;) {
        const int in = j % 3;
        if (threadIdx.x == 0) {
            s_cl = (long long)gc_aread(&c->und_cnt[in]);
            s_ch = (long long)gc_aread(&c->undh_cnt[in]);
        }
        __syncthreads();
        const long long cl = s_cl;
        long long ch = s_ch;
        const int* hl = L.undH[in];
        const bool hub_start = gc_hub_gate(g, c, j + 1, cl, hl, ch, L);
        if (cl + ch == 0 || cl > g.tail_lmax || ch > gc_tail_hmax(g)) break;
        ++j;
        const int out = j % 3, z = (j + 1) % 3;  // out was cleared by the sweep before
        __syncthreads();  // every thread has read hub_start before thread 0 moves it
        if (threadIdx.x == 0) {
            gc_st(&c->und_cnt[z], 0ull);
            gc_st(&c->undh_cnt[z], 0ull);
            gc_st(&c->sweeps, c->sweeps + 1);
            if (hub_start) gc_st(&c->hub_start, (long long)j);
        }
        gc_jp_sweep<NW>(g, L.undL[in], cl, 0, hl, ch, L.undL[out], &c->und_cnt[out], L.undH[out],
                    &c->undh_cnt[out], lsum, lnv, L.delta, &c->dcnt);
        __syncthreads();
    }
    if (threadIdx.x == 0) gc_st(&c->tail_last, (long long)j);
#if GC_SWEEP_STATS
    gc_stat_add<NW>(g, GC_K_SWEEP, lsum, lnv, scratch);
#endif
}

// ------------------------------------------------------------------------------------
// Asynchronous Jones-Plassmann (round 3): the rest of a round's JP chain after the first
// sweep (k_resolve) in ONE launch, with no grid barrier and no further host sweeps.
// Round 2 ran it as ~7 full-grid k_sweep launches plus the one-workgroup tail per round
// on R-MAT-24: a dependent chain of launches over a few thousand vertices each, ~110 us
// per round in launch floors.  Here every wave of a resident grid owns a
// static slice of the undecided lights and re-evaluates its pending ones from their
// cursors (lcur) pass after pass until they decide; then the wave's slice of the hubs
// (after EVERY light of the round has decided: the hub JP of gc_hubs.hip) likewise.
// No wave ever waits holding work another wave needs (it re-checks its own vertices), so
// the only dependence is JP's own: the lowest-rank undecided vertex of a candidate class
// can always decide, and states only move UND -> IN / OUT.
//   Visibility.  States another wave may read are stored agent-scope (sc1: written
// through, past this XCD's L2) and every load of them is an agent-scope load (sc1: past
// L1).  A stale read can only show UND -- the byte's candidate is fixed for the round and
// its state is final once set -- so staleness delays a decision, never changes it: the
// result is the same LFMIS as the sweeps'.  The hubs' wait for the lights is a counter:
// a wave publishes its decided lights with one atomic after `s_waitcnt vmcnt(0)` (its
// state and kill-flag stores have landed), and a hub wave polls the counter, then reads
// the kill flags with agent-scope loads.
//   Time budget.  A wave that finds the budget spent (wall clock, or another wave's
// flag) appends its pending vertices to the next undecided lists and leaves; the commit
// then sees them and the host runs ordinary sweeps (GC_H_SWEEPS), so a launch that was
// not fully resident, or a visibility stall, costs time and never a hang or a wrong
// colouring.  gc_stats.async_aborts counts such launches.
// ------------------------------------------------------------------------------------

#ifndef GC_KILL_DEFER
#define GC_KILL_DEFER 0  // k_sweep_async: light winners' hub kill flags raised in batches (round 6;
                         // measured slower: R-MAT-26 +5 ms, R-MAT-24 +-1, profiles/r06/q)
#endif
#define GC_KILL_BUF 256
struct GcAsyncLds {  // one wave's rows
    unsigned flag[GC_WAVE];
    int first[GC_WAVE];
    long long start[GC_WAVE];
    unsigned c6[GC_WAVE];
    int cv[GC_WAVE];
#if GC_KILL_DEFER
    int winv[GC_KILL_BUF];  // the wave's light winners whose hub kill flags are not raised yet
    int winc[GC_KILL_BUF];  //   and their colours
    int nwin;               //   (wave-uniform count)
#endif
};

// A light winner flags the hubs listing it that propose its colour (gc_hubs.hip): every
// entry of buf[0, nb) / col[0, nb), the wave walking their hub lists as one flat range.
__device__ void gc_async_kill_rows(GDev& g, const int* buf, const int* col, int nb, GcAsyncLds& s) {
    const int lane = gc_lane();
    for (int c0 = 0; c0 < nb; c0 += GC_WAVE) {
        const int v = c0 + lane < nb ? buf[c0 + lane] : -1;
        const int cv = c0 + lane < nb ? col[c0 + lane] : 0;
        int dh = 0;
        long long hs = 0;
        if (v >= 0) {
            hs = g.hin_rp[v];
            dh = (int)(g.hin_rp[v + 1] - hs);
        }
        gc_wave_sync();
        s.start[lane] = hs;
        s.cv[lane] = cv;
        const int hincl = gc_wave_incl_scan(dh);
        const int hexcl = hincl - dh;
        const int htotal = __shfl(hincl, GC_WAVE - 1, GC_WAVE);
        gc_wave_sync();
        gc_chunk_edges(
            g.hin_col, s.start, hexcl, htotal, [&](int hx) { return g.hk[hx]; },  // candidate field: fixed
            [&](int o, int hx, unsigned kh) {
                if ((kh >> 2) != (unsigned)s.cv[o]) return;
                if (!gc_ald32(g.hkill + hx)) gc_ast32(g.hkill + hx, 1u);
            });
        gc_wave_sync();
    }
}
#if GC_KILL_DEFER
// raise the kill flags of the buffered winners (the buffer is LDS: copied to registers first)
__device__ __forceinline__ void gc_async_kill_flush(GDev& g, GcAsyncLds& s) {
    const int nb = s.nwin;
    if (nb == 0) return;
    gc_async_kill_rows(g, s.winv, s.winc, nb, s);
    gc_wave_sync();
    if (gc_lane() == 0) s.nwin = 0;
    gc_wave_sync();
}
#endif

// One pass of a wave over its pending lights lst[0, np) (edge-balanced wave chunks, as
// gc_jp_sweep); the still-undecided ones are compacted to the front of lst (a chunk is
// read into registers before any of it is rewritten, and survivors only move down).
// Returns their number; `decided` counts the rest.
// Held lights (g.a_watch = R > 0, GC_A_WATCH): between full passes (every R-th), a light whose
// cursor entry -- its first pending entry at the last scan -- is still undecided with its
// candidate is kept without rescanning the rest of its range (an IN entry further on is seen
// at the next full pass; the decisions are the same).
// GC_LIGHT_LDS (round 6): a wave whose slice holds at most GC_LL_CAP lights keeps their words
// (vertex, cursor, low-row length, own byte, row start, candidate) in LDS after its first pass,
// so a later pass starts at its row reads: one LDS read instead of the list entry and the
// vertex's words, two dependent trips per 64-light chunk.
#ifndef GC_LIGHT_LDS
#define GC_LIGHT_LDS 1
#endif
#define GC_LL_CAP 256
struct GcLightLds {
    int v[GC_LL_CAP], lc[GC_LL_CAP], nl[GC_LL_CAP], cv[GC_LL_CAP];
    unsigned kv[GC_LL_CAP];
    long long rs[GC_LL_CAP];
};
// SRC = 1: the lights come from ll (else from lst and the vertex arrays); DST = 1: the
// survivors are compacted into ll (else into lst)
template <int SRC = 0, int DST = 0>
__device__ int gc_async_light_pass(GDev& g, int* lst, int np, GcAsyncLds& s, ull& decided, int pass,
                                   GcLightLds* ll = nullptr) {
    const int lane = gc_lane();
    const unsigned char* k8 = g.k8;
    const bool full_pass = g.a_watch <= 0 || pass % g.a_watch == 0;
    int nw = 0;
    for (int c0 = 0; c0 < np; c0 += GC_WAVE) {
        const int idx = c0 + lane;
        int v, lc, nl, cvv;
        unsigned kv, cv6;
        long long rs;
        if (SRC) {
            const bool in = idx < np;
            v = in ? ll->v[idx] : -1;
            lc = in ? ll->lc[idx] : 0;
            nl = in ? ll->nl[idx] : 0;
            kv = in ? ll->kv[idx] : 0xFFu;
            rs = in ? ll->rs[idx] : 0;
            cvv = in ? ll->cv[idx] : 0;
            cv6 = in ? gc_k8_cand(kv) : 0x100u;
        } else {
        v = idx < np ? lst[idx] : -1;
        if (v >= g.n) v = -1;  // never expected (a list entry out of range): skipped, not read through
        lc = v >= 0 ? g.lcur[v] : 0;
        nl = v >= 0 ? g.nlow[v] : 0;
        kv = v >= 0 ? (unsigned)k8[v] : 0xFFu;  // own byte: only this wave changes it
        rs = v >= 0 ? g.rp[v] : 0;
#if GC_HOIST_HIN
        const int cb0 = v >= 0 ? g.cand[v] : 0;
        cv6 = v >= 0 ? gc_k8_cand(kv) : 0x100u;
        cvv = (v >= 0 && cv6 == GC_K8_BIG) ? cb0 : (int)cv6;
#else
        cv6 = v >= 0 ? gc_k8_cand(kv) : 0x100u;
        cvv = (v >= 0 && cv6 == GC_K8_BIG) ? g.cand[v] : (int)cv6;
#endif
        }
        bool held = false;
        if (!full_pass && v >= 0 && lc < nl) {
            const int u0 = g.col[rs + lc];
            held = gc_jp_flag(g, u0, gc_ald8(k8 + u0), cv6, cvv) == 2u;
        }
        const int dl = (v >= 0 && !held) ? nl - lc : 0;
        s.flag[lane] = held ? 2u : 0u;
        s.first[lane] = held ? 0 : 0x7FFFFFFF;
        s.start[lane] = rs + lc;
        s.c6[lane] = cv6;
        s.cv[lane] = cvv;
        const int incl = gc_wave_incl_scan(dl);
        const int excl = incl - dl;
        const int total = __shfl(incl, GC_WAVE - 1, GC_WAVE);
        gc_wave_sync();
        gc_chunk_edges_at(
            g.col, s.start, excl, total, [&](int u) { return gc_ald8(k8 + u); },
            [&](int o, int u, unsigned ku, int slot) {
                const unsigned f = gc_jp_flag(g, u, ku, s.c6[o], s.cv[o]);
                if (f) atomicOr(&s.flag[o], f);
                if (f == 2u) atomicMin(&s.first[o], slot);
            });
        gc_wave_sync();
        unsigned nst = GC_JP_UND;
        bool pend = false;
        int nlc = lc;
        if (v >= 0) {
            const unsigned f = s.flag[lane];
            if (f & 1u) nst = GC_JP_OUT;
            else if (f & 2u) pend = true;
            else nst = GC_JP_IN;
            if (pend) {
                nlc = lc + s.first[lane];
                g.lcur[v] = nlc;  // (host sweeps resume from it after a give-up)
            } else {
                gc_ast8(g.k8 + v, (kv & ~3u) | nst);
            }
        }
        const ull pm = __ballot(pend);
        if (pend) {
            const int k = nw + __popcll(pm & gc_lanemask_lt());  // <= idx: survivors only move down
            if (DST) {
                ll->v[k] = v;
                ll->lc[k] = nlc;
                ll->nl[k] = nl;
                ll->kv[k] = kv;
                ll->rs[k] = rs;
                ll->cv[k] = cvv;
            } else {
                lst[k] = v;
            }
        }
        nw += __popcll(pm);
        decided += (ull)__popcll(__ballot(v >= 0 && !pend));
#if GC_KILL_DEFER
        // the wave's winners are buffered; their kill flags are raised in one flat walk when the
        // buffer fills and before the wave publishes its decided lights (only the hub phase
        // reads them, and it starts after every light's publication): a pass no longer waits
        // for each chunk's three dependent kill trips
        if (g.hub_w) {
            const bool iw = v >= 0 && nst == GC_JP_IN;
            const ull wmk = __ballot(iw);
            const int nwk = __popcll(wmk);
            if (nwk) {
                const int mycv = s.cv[lane];  // (a flush rewrites s.cv)
                if (s.nwin + nwk > GC_KILL_BUF) gc_async_kill_flush(g, s);
                const int b = s.nwin;
                gc_wave_sync();
                if (iw) {
                    const int k = b + __popcll(wmk & gc_lanemask_lt());
                    s.winv[k] = v;
                    s.winc[k] = mycv;
                }
                gc_wave_sync();
                if (lane == 0) s.nwin = b + nwk;
                gc_wave_sync();
            }
        }
#else
        if (g.hub_w) {  // a light winner flags the hubs listing it that propose its colour
            int dh = 0;
            long long hs = 0;
            if (nst == GC_JP_IN) {
                hs = g.hin_rp[v];
                dh = (int)(g.hin_rp[v + 1] - hs);
            }
            gc_wave_sync();
            s.start[lane] = hs;
            const int hincl = gc_wave_incl_scan(dh);
            const int hexcl = hincl - dh;
            const int htotal = __shfl(hincl, GC_WAVE - 1, GC_WAVE);
            gc_wave_sync();
            gc_chunk_edges(
                g.hin_col, s.start, hexcl, htotal, [&](int hx) { return g.hk[hx]; },  // candidate field: fixed
                [&](int o, int hx, unsigned kh) {
                    if ((kh >> 2) != (unsigned)s.cv[o]) return;
                    if (!gc_ald32(g.hkill + hx)) gc_ast32(g.hkill + hx, 1u);
                });
        }
#endif
        gc_wave_sync();
    }
    return nw;
}

#ifdef GC_A_PROF
// (diagnostic build, -DGC_A_PROF: per round, where k_sweep_async's time goes -- the light
// phase, the wait for the last light, the hub phase -- and the passes each took; dumped by
// the engine at the end of the colouring, GC_A_PROF_OUT=path)
#define GC_A_PROF_ROUNDS 4096
#define GC_A_PROF_K 16
__device__ ull gc_aprof[GC_A_PROF_ROUNDS][GC_A_PROF_K];
#endif

// One pass of a wave over its pending hubs hl[0, nh), GC_HUB_NG at a time (a 16-lane
// group each): the resumable scan of gc_hub_scan_groups, with agent-scope loads of the
// hub mirror and the kill flags and agent-scope stores of the decisions.  Pending hubs
// are compacted to the front of hl; returns their number.
// The hubs' own words (k8, cand, hid, then hkill, hlow_rp, hpc, hcur, hlen) are loaded for
// 64 hubs at once, one per lane, and handed to the groups by shuffles (GC_HUB_PREFETCH, the
// default; as the host sweeps' gc_hub_scan_groups): a group that loaded its hub's words
// itself paid three dependent trips per hub before its row scan, ~16 times per 64 hubs.
// (The kill flags are final during the hub phase: every light of the round has decided
// before it starts.)  Entries are read a batch at a time, and survivors only move down, so
// the compaction never overwrites an entry not yet read.
#ifndef GC_HUB_PREFETCH
#define GC_HUB_PREFETCH 1
#endif
template <int NG = GC_HUB_NG>
__device__ int gc_async_hub_pass(GDev& g, int* hl, int nh) {
    constexpr int GS = GC_WAVE / NG;
    const int lane = gc_lane();
    const int grp = lane / GS, li = lane % GS;
    const ull gmask = GS >= GC_WAVE ? ~0ull : ((1ull << (GS % GC_WAVE)) - 1ull) << (grp * GS);
    int nw = 0;
#if GC_HUB_PREFETCH
    for (int b0 = 0; b0 < nh; b0 += GC_WAVE) {
    const int bn = nh - b0 < GC_WAVE ? nh - b0 : GC_WAVE;
    const int pv = lane < bn ? hl[b0 + lane] : -1;
    const unsigned pkv = pv >= 0 ? (unsigned)g.k8[pv] : 0u;  // own byte
    const int pcb = pv >= 0 ? g.cand[pv] : 0;                // read with k8: used when the candidate is >= 62
    const int px = pv >= 0 ? g.hid[pv] : -1;                 // every heavy proposer is a hub while the hub JP is on
    const int pcv = gc_k8_cand(pkv) == GC_K8_BIG ? pcb : (int)gc_k8_cand(pkv);
    const int pkill = px >= 0 ? (int)gc_ald32(g.hkill + px) : 0;
    long long pbase = 0;
    int pfull = 0, pcur = 0, phc0 = 1, phs = 0;
    if (px >= 0) {
        pbase = g.hlow_rp[px];
        pfull = (int)(g.hlow_rp[px + 1] - pbase);
        pcur = g.hpc[px];
        phc0 = g.hcur[px];
        phs = g.hlen[px];
    }
    for (int j0 = 0; j0 < bn; j0 += NG) {
        const int j = j0 + grp;
        const bool has = j < bn;
        const int jj = has ? j : 0;  // every lane takes part in every shuffle
        const int vs = __shfl(pv, jj, GC_WAVE);
        const int v = has ? vs : -1;
        const unsigned kv = (unsigned)__shfl((int)pkv, jj, GC_WAVE);
        const int cv = __shfl(pcv, jj, GC_WAVE);
        const int xs = __shfl(px, jj, GC_WAVE);
        const int x = has ? xs : -1;
        const int ks = __shfl(pkill, jj, GC_WAVE);  // not under a condition: a lane left out of a
        const bool kill = x >= 0 && ks != 0;         // shuffle reads back nothing from its source
        const long long base = __shfl(pbase, jj, GC_WAVE);
        const int full = __shfl(pfull, jj, GC_WAVE);
        const int cursor = __shfl(pcur, jj, GC_WAVE);
        const int hc0 = __shfl(phc0, jj, GC_WAVE);
        const int hstart = __shfl(phs, jj, GC_WAVE);
#else
    for (int j0 = 0; j0 < nh; j0 += NG) {
        const int j = j0 + grp;
        const int v = j < nh ? hl[j] : -1;
        const unsigned kv = v >= 0 ? (unsigned)g.k8[v] : 0u;  // own byte
        const int cv = v >= 0 ? (gc_k8_cand(kv) == GC_K8_BIG ? g.cand[v] : (int)gc_k8_cand(kv)) : 0;
        const int x = v >= 0 ? g.hid[v] : -1;  // every heavy proposer is a hub while the hub JP is on
        const bool kill = x >= 0 && gc_ald32(g.hkill + x) != 0u;
        long long base = 0;
        int full = 0, cursor = 0, hc0 = 1, hstart = 0;
        if (x >= 0) {
            base = g.hlow_rp[x];
            full = (int)(g.hlow_rp[x + 1] - base);
            cursor = g.hpc[x];
            hc0 = g.hcur[x];
            hstart = g.hlen[x];
        }
#endif
        const bool act = x >= 0 && !kill;  // group-uniform
        const bool first = hc0 == 0;
        int pos = first ? hstart : cursor;
        bool out = false, prefix = act && first;
        int block = -1, nstart = full;
        const int* __restrict__ row = g.hlow_col + base;
        for (;;) {
            const bool run = act && !out && block < 0 && pos < full;
            if (!__ballot(run)) break;
            int u[GC_HUB_UNR];
#pragma unroll
            for (int k = 0; k < GC_HUB_UNR; ++k) {
                const int e = pos + k * GS + li;
                u[k] = (run && e < full) ? row[e] : -1;
            }
            unsigned ku[GC_HUB_UNR];
#pragma unroll
            for (int k = 0; k < GC_HUB_UNR; ++k) ku[k] = u[k] >= 0 ? gc_ald32(g.hk + u[k]) : GC_HK_COLOURED;
            unsigned fl[GC_HUB_UNR];
#pragma unroll
            for (int k = 0; k < GC_HUB_UNR; ++k) fl[k] = ku[k] != GC_HK_COLOURED ? gc_jp_flag_h(g, u[k], ku[k], 0u, cv) : 0u;
#pragma unroll
            for (int k = 0; k < GC_HUB_UNR; ++k) {
                if (__ballot(fl[k] == 1u) & gmask) out = true;
                const ull mb = __ballot(fl[k] == 2u) & gmask;
                if (mb && block < 0) block = pos + k * GS + __builtin_ctzll(mb >> (grp * GS));
                const ull ml = __ballot(u[k] >= 0 && ku[k] != GC_HK_COLOURED) & gmask;
                if (prefix && ml) {  // first non-coloured entry: the end of the coloured prefix
                    nstart = pos + k * GS + __builtin_ctzll(ml >> (grp * GS));
                    prefix = false;
                }
            }
            if (run) pos += GC_HUB_UNR * GS;
        }
        unsigned f = kill ? 1u : 0u;
        if (act) f = out ? 1u : (block >= 0 ? 2u : 0u);
        const bool lead = li == 0 && x >= 0;
#ifdef GC_A_PROF
        if (lead && act && g.ctl->round < GC_A_PROF_ROUNDS) {
            ull* r = gc_aprof[g.ctl->round];
            const int p0 = first ? hstart : cursor;
            const ull sc = (ull)(std::min(pos, full) - p0);
            atomicAdd(r + 12, sc);
            atomicMax(r + 13, sc);
            if (f == 0u) atomicAdd(r + 14, 1ull);
            if (first) atomicAdd(r + 15, (ull)(full - hstart));
        }
#endif
        if (lead && act) {
            if (first) {
                g.hcur[x] = 1;
                if (nstart > hstart) g.hlen[x] = nstart;
            }
            if (!out && block >= 0) g.hpc[x] = block;
        }
        if (lead && f != 2u) {
            const unsigned st = (f & 1u) ? GC_JP_OUT : GC_JP_IN;
            gc_ast8(g.k8 + v, (kv & ~3u) | st);
            gc_ast32(g.hk + x, gc_hk((unsigned)cv, st));
        }
        const bool pend = lead && f == 2u;
        const ull pm = __ballot(pend);
        if (pend) hl[nw + __popcll(pm & gc_lanemask_lt())] = v;
        nw += __popcll(pm);
    }
#if GC_HUB_PREFETCH
    }
#endif
    return nw;
}

// the launch's budget is spent, or another wave found it so (wave-uniform)
__device__ __forceinline__ bool gc_async_stop(DevCtl* c, int par, ull t0, long long budget) {
    int stop = 0;
    if (gc_lane() == 0) {
        stop = __hip_atomic_load(&c->async_abort[par], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!stop && (long long)(wall_clock64() - t0) > budget) {
            stop = 1;
            if (atomicCAS(&c->async_abort[par], 0, 1) == 0) atomicAdd(&c->async_aborts, 1ull);
        }
    }
    return __shfl(stop, 0, GC_WAVE) != 0;
}

// pending entries src[0, cnt) of a wave that gave up -> the next undecided list
__device__ __forceinline__ void gc_async_spill(const int* src, int cnt, int* out, ull* out_cnt) {
    if (cnt <= 0) return;
    ull base = 0;
    if (gc_lane() == 0) base = atomicAdd(out_cnt, (ull)cnt);
    base = __shfl(base, 0, GC_WAVE);
    for (int i = gc_lane(); i < cnt; i += GC_WAVE) out[base + i] = src[i];
}


// The hub phase of a wave whose slice holds at most 64 hubs (every small round: the slices
// are GC_HUB_NG hubs), with each hub's words kept in ITS lane's registers across passes
// (round 6; GC_HUB_REG, the default).  gc_async_hub_pass reloads a hub's words -- the list
// entry, then k8 / cand / hid, then hkill / hlow_rp / hpc / hcur / hlen -- in every pass:
// three dependent trips before each pass's row scan, ~12 passes a round.  Here they are
// loaded once, and a hub whose scan stopped at an undecided same-candidate entry (the
// blocker, its cursor) WATCHES that one entry: a later pass gathers the blockers' hub words
// for all of the wave's pending hubs in one trip, and only a hub whose blocker has decided
// resumes its scan (from the blocker, re-read, as gc_async_hub_pass resumes from the cursor).
// The decisions are the resumable scan's (same cursor, same prefix, same flags); the cursor
// and prefix words are stored as that pass stores them, so host sweeps after a give-up
// resume from them.  Returns the hubs still pending when the wave stops (spilled by it).
#ifndef GC_HUB_WIN
#define GC_HUB_WIN 1
#endif
#ifndef GC_HUB_WIDE
#define GC_HUB_WIDE 1
#endif
#ifndef GC_HUB_REG
#define GC_HUB_REG 1  // R-MAT-24 146.2 -> 143.1 ms, R-MAT-26 383.4 -> 379.3 without the watch (profiles/r06/r)
#endif
#ifndef GC_HUB_WATCH
#define GC_HUB_WATCH 0  // the watched blocker: slower (a blocker that decided costs a trip more; profiles/r06/r)
#endif
template <int NG = GC_HUB_NG>
__device__ int gc_async_hubs_reg(GDev& g, const int* src, int nh0, DevCtl* c, int par, ull t0, long long budget,
                                 int* spill, ull* spill_cnt, ull* hpass_out, int* s_own) {
    constexpr int GS = GC_WAVE / NG;
    const int lane = gc_lane();
    const int grp = lane / GS, li = lane % GS;
    const ull gmask = GS >= GC_WAVE ? ~0ull : ((1ull << (GS % GC_WAVE)) - 1ull) << (grp * GS);
    // this lane's hub (lane j = entry j of the slice)
    const int v = lane < nh0 ? src[lane] : -1;
    const unsigned kv = v >= 0 ? (unsigned)g.k8[v] : 0u;  // own byte
    const int cb = v >= 0 ? g.cand[v] : 0;
    const int x = v >= 0 ? g.hid[v] : -1;  // every heavy proposer is a hub while the hub JP is on
    const int cv = gc_k8_cand(kv) == GC_K8_BIG ? cb : (int)gc_k8_cand(kv);
    bool kill = false;
    long long base = 0;
    int full = 0, pos = 0, hstart = 0;
    bool first = false;
    if (x >= 0) {
        kill = gc_ald32(g.hkill + x) != 0u;  // final in the hub phase
        base = g.hlow_rp[x];
        full = (int)(g.hlow_rp[x + 1] - base);
        const int cursor = g.hpc[x];
        first = g.hcur[x] == 0;
        hstart = g.hlen[x];
        pos = first ? hstart : cursor;
    }
    int ublk = -1;            // the watched blocker (hub index) once a scan stopped at one
    bool pend = x >= 0;       // undecided (entries that are no hub are dropped, as in gc_async_hub_pass)
    ull hpass = 0;
    int idle = 0;
    for (;;) {
        ++hpass;
        // the watched blockers of every pending hub in one trip: still undecided with the
        // hub's candidate -> the hub stays blocked without reading its row
        bool scan = pend;
        if (GC_HUB_WATCH && pend && !kill && ublk >= 0) {
            const unsigned kb = gc_ald32(g.hk + ublk);
            if (kb != GC_HK_COLOURED && gc_jp_flag_h(g, ublk, kb, 0u, cv) == 2u) scan = false;
        }
        const ull sm = __ballot(scan);
        const int rk = __popcll(sm & gc_lanemask_lt());  // this lane's rank among the scanning hubs
        const int ns = __popcll(sm);
        int decided = 0;
        gc_wave_sync();
        if (scan) s_own[rk] = lane;  // rank -> owner lane (LDS row of this wave)
        gc_wave_sync();
        for (int j0 = 0; j0 < ns; j0 += NG) {
            // group grp takes the scanning hub of rank j0 + grp (its owner lane ol)
            const int want = j0 + grp;
            const bool has = want < ns;
            const int ol = has ? s_own[want] : 0;
            const int hv = __shfl(v, ol, GC_WAVE);
            const int hcv = __shfl(cv, ol, GC_WAVE);
            const int hkill = __shfl((int)kill, ol, GC_WAVE);
            const long long hbase = __shfl(base, ol, GC_WAVE);
            const int hfull = __shfl(full, ol, GC_WAVE);
            const int hpos = __shfl(pos, ol, GC_WAVE);
            const int hfirst = __shfl((int)first, ol, GC_WAVE);
            (void)hv;
            const bool act = has && !hkill;  // group-uniform
            int p = hpos;
            bool out = false, prefix = act && hfirst;
            int block = -1, nstart = hfull, ub = -1;
            const int* __restrict__ row = g.hlow_col + hbase;
            for (;;) {
                const bool run = act && !out && block < 0 && p < hfull;
                if (!__ballot(run)) break;
                int u[GC_HUB_UNR];
#pragma unroll
                for (int k = 0; k < GC_HUB_UNR; ++k) {
                    const int e = p + k * GS + li;
                    u[k] = (run && e < hfull) ? row[e] : -1;
                }
                unsigned ku[GC_HUB_UNR];
#pragma unroll
                for (int k = 0; k < GC_HUB_UNR; ++k) ku[k] = u[k] >= 0 ? gc_ald32(g.hk + u[k]) : GC_HK_COLOURED;
#pragma unroll
                for (int k = 0; k < GC_HUB_UNR; ++k) {
                    const unsigned fl = ku[k] != GC_HK_COLOURED ? gc_jp_flag_h(g, u[k], ku[k], 0u, hcv) : 0u;
                    if (__ballot(fl == 1u) & gmask) out = true;
                    const ull mb = __ballot(fl == 2u) & gmask;
                    const int bl = mb ? __ffsll((long long)mb) - 1 : lane;
                    const int bu = __shfl(u[k], bl, GC_WAVE);  // every lane takes part
                    if (mb && block < 0) {
                        block = p + k * GS + (bl - grp * GS);
                        ub = bu;
                    }
                    const ull ml = __ballot(u[k] >= 0 && ku[k] != GC_HK_COLOURED) & gmask;
                    if (prefix && ml) {  // first non-coloured entry: the end of the coloured prefix
                        nstart = p + k * GS + __builtin_ctzll(ml >> (grp * GS));
                        prefix = false;
                    }
                }
                if (run) p += GC_HUB_UNR * GS;
            }
            const unsigned f = hkill ? 1u : (out ? 1u : (block >= 0 ? 2u : 0u));
            // back to the owner lanes: lane r of rank j0 + q reads group q's leader
            const bool mine = scan && rk >= j0 && rk < j0 + NG;
            const int src_l = mine ? (rk - j0) * GS : lane;
            const unsigned rf = (unsigned)__shfl((int)f, src_l, GC_WAVE);
            const int rblock = __shfl(block, src_l, GC_WAVE);
            const int rub = __shfl(ub, src_l, GC_WAVE);
            const int rns = __shfl(nstart, src_l, GC_WAVE);
            const int ract = __shfl((int)act, src_l, GC_WAVE);
            if (mine) {
                if (ract) {
                    if (first) {
                        g.hcur[x] = 1;
                        if (rns > hstart) g.hlen[x] = rns;
                        first = false;
                    }
                    if (rf == 2u) {
                        g.hpc[x] = rblock;
                        pos = rblock;
                        ublk = rub;
                    }
                }
                if (rf != 2u) {
                    const unsigned st = (rf & 1u) ? GC_JP_OUT : GC_JP_IN;
                    gc_ast8(g.k8 + v, (kv & ~3u) | st);
                    gc_ast32(g.hk + x, gc_hk((unsigned)cv, st));
                    pend = false;
                    decided = 1;
                }
            }
        }
        if (!__ballot(pend)) break;
        if (gc_async_stop(c, par, t0, budget)) {
            const ull pm = __ballot(pend);
            ull b = 0;
            if (lane == 0) b = atomicAdd(spill_cnt, (ull)__popcll(pm));
            b = __shfl(b, 0, GC_WAVE);
            if (pend) spill[b + __popcll(pm & gc_lanemask_lt())] = v;
            *hpass_out = hpass;
            return __popcll(pm);
        }
        if (!__ballot(decided)) {
            if (++idle > 2) __builtin_amdgcn_s_sleep(2);
        } else {
            idle = 0;
        }
    }
    *hpass_out = hpass;
    return 0;
}

// One hub per wave (GC_HUB_WIDE), its words in registers and its row window too (GC_HUB_WIN,
// round 6): a scan that stopped at an undecided same-candidate entry keeps the 512 entries it
// loaded (8 a lane), and the next pass re-gathers their hub words from the window's start --
// the entries before the blocker were coloured, OUT or of another candidate, final within the
// launch, so they read as not blocking again -- one dependent trip a pass instead of two
// (the row entries, then their hub words).  The decisions and the stored cursor / prefix are
// the resumable scan's.
__device__ void gc_async_hub_win(GDev& g, const int* src, int nh0, DevCtl* c, int par, ull t0, long long budget,
                                 int* spill, ull* spill_cnt, ull* hpass_out) {
    constexpr int STEP = GC_HUB_UNR * GC_WAVE;
    const int lane = gc_lane();
    *hpass_out = 0;
    if (nh0 <= 0) return;
    const int v = src[0];
    const unsigned kv = (unsigned)g.k8[v];  // own byte
    const int cb = g.cand[v];
    const int x = g.hid[v];
    if (x < 0) return;  // no hub (cannot happen while the hub JP is on): dropped, as gc_async_hub_pass does
    const int cv = gc_k8_cand(kv) == GC_K8_BIG ? cb : (int)gc_k8_cand(kv);
    const bool kill = gc_ald32(g.hkill + x) != 0u;
    const long long base = g.hlow_rp[x];
    const int full = (int)(g.hlow_rp[x + 1] - base);
    const int cursor = g.hpc[x];
    bool first = g.hcur[x] == 0;
    const int hstart = g.hlen[x];
    const int* __restrict__ row = g.hlow_col + base;
    int pos = first ? hstart : cursor;
    int u[GC_HUB_UNR];
    int wlo = -1;  // the window holds row[wlo + k * 64 + lane] in u[k] (or -1 past the row)
    ull hpass = 0;
    int idle = 0;
    unsigned f = 1u;  // killed: OUT
    if (!kill) {
        for (;;) {
            ++hpass;
            bool out = false, prefix = first;
            int block = -1, nstart = full;
            int p = pos;
            while (!out && block < 0 && p < full) {
                if (wlo < 0 || p < wlo || p >= wlo + STEP) {  // a new window from p
                    wlo = p;
#pragma unroll
                    for (int k = 0; k < GC_HUB_UNR; ++k) {
                        const int e = wlo + k * GC_WAVE + lane;
                        u[k] = e < full ? row[e] : -1;
                    }
                }
                unsigned ku[GC_HUB_UNR];
#pragma unroll
                for (int k = 0; k < GC_HUB_UNR; ++k) {
                    const int e = wlo + k * GC_WAVE + lane;
                    ku[k] = (u[k] >= 0 && e >= p) ? gc_ald32(g.hk + u[k]) : GC_HK_COLOURED;
                }
#pragma unroll
                for (int k = 0; k < GC_HUB_UNR; ++k) {
                    const unsigned fl = ku[k] != GC_HK_COLOURED ? gc_jp_flag_h(g, u[k], ku[k], 0u, cv) : 0u;
                    if (__ballot(fl == 1u)) out = true;
                    const ull mb = __ballot(fl == 2u);
                    if (mb && block < 0) block = wlo + k * GC_WAVE + __builtin_ctzll(mb);
                    const ull ml = __ballot(u[k] >= 0 && ku[k] != GC_HK_COLOURED);
                    if (prefix && ml) {  // first non-coloured entry: the end of the coloured prefix
                        nstart = wlo + k * GC_WAVE + __builtin_ctzll(ml);
                        prefix = false;
                    }
                }
                if (!out && block < 0) p = wlo + STEP;
            }
            if (lane == 0 && first) {
                g.hcur[x] = 1;
                if (nstart > hstart) g.hlen[x] = nstart;
            }
            first = false;
            f = out ? 1u : (block >= 0 ? 2u : 0u);
            if (f != 2u) break;
            if (lane == 0) g.hpc[x] = block;
            pos = block;
            if (gc_async_stop(c, par, t0, budget)) {
                ull b = 0;
                if (lane == 0) b = atomicAdd(spill_cnt, 1ull);
                b = __shfl(b, 0, GC_WAVE);
                if (lane == 0) spill[b] = v;
                *hpass_out = hpass;
                return;
            }
            if (++idle > 2) __builtin_amdgcn_s_sleep(2);
        }
    }
    if (lane == 0) {
        const unsigned st = (f & 1u) ? GC_JP_OUT : GC_JP_IN;
        gc_ast8(g.k8 + v, (kv & ~3u) | st);
        gc_ast32(g.hk + x, gc_hk((unsigned)cv, st));
    }
    *hpass_out = hpass;
}

// The launch after sweep S (k_resolve = 0, or the last host sweep): reads slot S % 3,
// spills to slot (S + 1) % 3 (cleared by sweep S), clears slot (S + 2) % 3 and sets
// tail_last = S + 1, the slot the commit checks -- exactly what a tail that ran one more
// sweep leaves.  `par` alternates per launch (the counters of the next launch are zeroed
// here); `budget` is in wall-clock ticks.  (Round 3's variant that also made the round's
// first sweep, in place of k_resolve, measured R-MAT-24 172.7 -> 190.4 ms in round 4,
// profiles/r04/c: removed.)
__global__ void __launch_bounds__(GC_BLOCK) k_sweep_async(GDev g, GLists L, int S, int par, long long budget,
                                                          int lds_lights) {
    DevCtl* c = g.ctl;
    if (budget < 0) {  // residency probe (gcl_sweep_async_resident)
        gc_residency_probe(c);
        return;
    }
    if (c->halt) return;
    if (c->core_round == c->round) return;  // k_hub_core decided this round's hubs (gc_core.hip)
    __shared__ GcAsyncLds s_w[GC_WAVES_PER_BLOCK];
    const int w = threadIdx.x / GC_WAVE;
    const long long j = S;
    const int in = (int)(j % 3), out = (int)((j + 1) % 3), z = (int)((j + 2) % 3);
    const long long cl = (long long)c->und_cnt[in];
    // hubs already started by an earlier sweep of the round: their undecided list; else every
    // hub proposer, once the lights have converged.  (hub_start moves during the launch only
    // from "not started" to S + 1 > S: every reader takes the same branch.)
    const bool started = g.hub_w && __hip_atomic_load(&c->hub_start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= j;
    const int* hsrc = started ? L.undH[in] : L.heavy;
    const long long ch = g.hub_w ? (long long)(started ? c->undh_cnt[in] : c->heavy_cnt) : 0ll;
    if (cl > g.n || ch > g.n || cl < 0) {  // never expected: report (the host turns it into an error), touch nothing
        if (blockIdx.x == 0 && threadIdx.x == 0) __hip_atomic_store(&c->loop_err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        c->und_cnt[z] = 0;
        c->undh_cnt[z] = 0;
        c->tail_last = j + 1;
        if (cl + ch > 0) c->sweeps += 1;
        c->async_done[par ^ 1] = 0;
        c->async_abort[par ^ 1] = 0;
        if (!started && ch > 0 && cl == 0) gc_st(&c->hub_start, j + 1);
    }
    const ull t0 = wall_clock64();
    // the budget grows with the launch's lists (20 ns of wall clock per light, 80 per hub): a
    // give-up is for stalls, not for big rounds (R-MAT-28's lists reach ~10^7)
    budget += 2 * (cl + 4 * ch);
    const long long W = (long long)gridDim.x * GC_WAVES_PER_BLOCK;
    const long long wid = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w;
    bool stop = false;
#ifdef GC_A_PROF
    ull* aprof = (gc_lane() == 0 && c->round < GC_A_PROF_ROUNDS) ? gc_aprof[c->round] : nullptr;
    if (aprof && wid == 0) {
        aprof[5] = (ull)cl;
        aprof[6] = (ull)ch;
    }
#endif
    // lights: the wave's static slice of the list, compacted in place pass after pass
    {
        const long long la = cl * wid / W, lb = cl * (wid + 1) / W;
        int np = (int)(lb - la);
#ifdef GC_A_PROF
        if (aprof && np > 0) atomicMax(aprof + 9, (ull)np);
#endif
        int* lst = L.undL[in] + la;
        ull decided = 0;
        int idle = 0, lpass = 0;
#if GC_KILL_DEFER
        if (gc_lane() == 0) s_w[w].nwin = 0;
        gc_wave_sync();
#endif
#if GC_LIGHT_LDS
        extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
        GcLightLds* s_ll = reinterpret_cast<GcLightLds*>(s_dyn);
        const bool lds = lds_lights && np <= GC_LL_CAP;
#else
        (void)lds_lights;
        const bool lds = false;
        (void)lds;
#endif
        while (np > 0) {
            const int before = np;
#if GC_LIGHT_LDS
            if (lds) np = lpass == 0 ? gc_async_light_pass<0, 1>(g, lst, np, s_w[w], decided, ++lpass, &s_ll[w])
                                     : gc_async_light_pass<1, 1>(g, lst, np, s_w[w], decided, ++lpass, &s_ll[w]);
            else
#endif
            np = gc_async_light_pass(g, lst, np, s_w[w], decided, ++lpass);
            if (np == 0) break;
            if ((stop = gc_async_stop(c, par, t0, budget))) break;
            if (np == before) {
#if GC_KILL_DEFER
                // waiting on other waves: raise the buffered winners' kill flags meanwhile
                if (g.hub_w && s_w[w].nwin > 0) {
                    gc_async_kill_flush(g, s_w[w]);
                    continue;
                }
#endif
                if (++idle > 2) __builtin_amdgcn_s_sleep(2);
            } else {
                idle = 0;
            }
        }
        if (stop) {
#if GC_LIGHT_LDS
            if (lds && lpass > 0) {  // the survivors are in LDS
                gc_wave_sync();
                for (int i = gc_lane(); i < np; i += GC_WAVE) lst[i] = s_ll[w].v[i];
                gc_wave_sync();
            }
#endif
            gc_async_spill(lst, np, L.undL[out], &c->und_cnt[out]);
        }
#if GC_KILL_DEFER
        if (g.hub_w) gc_async_kill_flush(g, s_w[w]);  // before the publication below
#endif
#ifdef GC_A_PROF
        if (aprof && lpass > 0) {
            atomicMax(aprof + 0, wall_clock64() - t0);
            atomicMax(aprof + 3, (ull)lpass);
            atomicAdd(aprof + 7, (ull)lpass);
            atomicAdd(aprof + 8, 1ull);
        }
#endif
        if (decided) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // its state and kill-flag stores have landed
            if (gc_lane() == 0) {
                const ull old = atomicAdd(&c->async_done[par], decided);
                if (old + decided == (ull)cl && ch > 0 && !started) gc_st(&c->hub_start, j + 1);
            }
        }
    }
    if (ch == 0) return;
    // hubs: the wave's slice (GC_HUB_NG at least), copied to slot z (the source lists stay
    // intact: the commit walks L.heavy) and compacted there
    // GC_HUB_WIDE (round 6): while the hubs fit one per wave (every small round), each wave
    // takes ONE hub and scans its row with all 64 lanes (512 entries a step): a round's first
    // evaluation walks ~280 entries past the coloured prefix (coloured hubs interleave with
    // the uncoloured ones in rank order), 4-5 steps for a 16-lane group, one for a wave
    const bool wide = GC_HUB_WIDE && ch <= W;
    const long long per = wide ? 1ll : std::max<long long>(GC_HUB_NG, (ch + W - 1) / W);
    const long long ha = wid * per;
    if (ha >= ch) return;
    const int nh0 = (int)(std::min(ch, ha + per) - ha);
    const int* src = hsrc + ha;
    if (!stop && cl > 0) {  // wait for every light of the round
        int st = 0;
        if (gc_lane() == 0) {
            while (__hip_atomic_load(&c->async_done[par], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (ull)cl) {
                st = __hip_atomic_load(&c->async_abort[par], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (!st && (long long)(wall_clock64() - t0) > budget) {
                    st = 1;
                    if (atomicCAS(&c->async_abort[par], 0, 1) == 0) atomicAdd(&c->async_aborts, 1ull);
                }
                if (st) break;
                __builtin_amdgcn_s_sleep(4);
            }
        }
        stop = __shfl(st, 0, GC_WAVE) != 0;
    }
#ifdef GC_A_PROF
    if (aprof) atomicMax(aprof + 1, wall_clock64() - t0);
#endif
    if (stop) {
        // hubs unevaluated: always listed.  The lights may still converge after this wave
        // gave up (the last light wave publishing late), and then hub_start = S + 1 and every
        // undecided hub must be on the list; if they never converge, the host's sweeps start
        // the hubs from L.heavy themselves and ignore this list (gc_hub_gate)
        gc_async_spill(src, nh0, L.undH[out], &c->undh_cnt[out]);
        return;
    }
    if (GC_HUB_REG && nh0 <= GC_WAVE) {  // the slice's words in registers (gc_async_hubs_reg)
        ull hp = 0;
        if (wide && GC_HUB_WIN)  // one hub, all 64 lanes on its row, the row window kept
            gc_async_hub_win(g, src, nh0, c, par, t0, budget, L.undH[out], &c->undh_cnt[out], &hp);
        else if (wide)  // one hub, all 64 lanes on its row
            gc_async_hubs_reg<1>(g, src, nh0, c, par, t0, budget, L.undH[out], &c->undh_cnt[out], &hp, s_w[w].first);
        else
            gc_async_hubs_reg<GC_HUB_NG>(g, src, nh0, c, par, t0, budget, L.undH[out], &c->undh_cnt[out], &hp,
                                         s_w[w].first);
#ifdef GC_A_PROF
        if (aprof) {
            atomicMax(aprof + 2, wall_clock64() - t0);
            atomicMax(aprof + 4, hp);
            atomicAdd(aprof + 10, hp);
            atomicMax(aprof + 11, (ull)nh0);
        }
#endif
        return;
    }
    int* hl = L.undH[z] + ha;
    for (int i = gc_lane(); i < nh0; i += GC_WAVE) hl[i] = src[i];
    gc_wave_sync();
    int nh = nh0, idle = 0;
#ifdef GC_A_PROF
    ull hpass = 0;
#endif
    while (nh > 0) {
        const int before = nh;
#ifdef GC_A_PROF
        ++hpass;
#endif
        nh = wide ? gc_async_hub_pass<1>(g, hl, nh) : gc_async_hub_pass<GC_HUB_NG>(g, hl, nh);
        if (nh == 0) break;
        if ((stop = gc_async_stop(c, par, t0, budget))) break;
        if (nh == before) {
            if (++idle > 2) __builtin_amdgcn_s_sleep(2);
        } else {
            idle = 0;
        }
    }
    if (stop) gc_async_spill(hl, nh, L.undH[out], &c->undh_cnt[out]);
#ifdef GC_A_PROF
    if (aprof) {
        atomicMax(aprof + 2, wall_clock64() - t0);
        atomicMax(aprof + 4, hpass);
        atomicAdd(aprof + 10, hpass);
        atomicMax(aprof + 11, (ull)nh0);
    }
#endif
}

// ------------------------------------------------------------------------------------
// commit (color_node + join, coloring.py:37-41, 114-127) fused with the frontier push,
// and the end-of-round bookkeeping (last workgroup).
// ------------------------------------------------------------------------------------

// GC_CHECKS: record the first out-of-range value (code, a, b, c) and report it (loop_err 3)
__device__ __forceinline__ void gc_dbg(DevCtl* c, long long code, long long a, long long b, long long cc) {
    if (atomicCAS(reinterpret_cast<ull*>(&c->dbg[0]), 0ull, (ull)code) == 0ull) {
        c->dbg[1] = a;
        c->dbg[2] = b;
        c->dbg[3] = cc;
        __hip_atomic_store(&c->loop_err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// big-round push (k_commit / k_commit_big, mark mode): in-neighbour x of a winner joins the
// next frontier.  GC_MARK_CHECK (round 6): only when its claim bit is clear -- coloured or
// already-frontier vertices (most of a big round's in-neighbours) need no mark, and a read of
// the 1/8-byte-per-vertex claim bitmap is cheaper than a random partial-line byte store
#ifndef GC_MARK_CHECK
#define GC_MARK_CHECK 1
#endif
__device__ __forceinline__ void gc_mark(const GDev& g, int x) {
    if (GC_MARK_CHECK && ((g.inF[x >> 5] >> (x & 31)) & 1u)) return;
    g.mark[x] = 1;
}
__device__ __forceinline__ bool gc_claim(unsigned* inF, int x) {
    const unsigned bit = 1u << (x & 31);
    if (inF[x >> 5] & bit) return false;
    return !(atomicOr(&inF[x >> 5], bit) & bit);
}
__device__ __forceinline__ bool gc_claim_direct(unsigned* inF, int x) {
    const unsigned bit = 1u << (x & 31);
    return !(atomicOr(&inF[x >> 5], bit) & bit);
}
#ifndef GC_CSLOTS
#define GC_CSLOTS 2
#endif
#ifndef GC_PREFETCH_ROW
#define GC_PREFETCH_ROW 1
#endif
#ifndef GC_COMMIT_HUB_LANES
#define GC_COMMIT_HUB_LANES 1  // k_commit: a run of heavy entries per wave, one per lane (round 6)
#endif
#ifndef GC_CB_UNR
#define GC_CB_UNR 1  // k_commit_big: entries a thread per step (round 6: 4 measured slower, R-MAT-24 +2 ms,
                     // R-MAT-26 +3.9 ms, profiles/r06/u)
#endif
#ifndef GC_COMMIT_FLAT
#define GC_COMMIT_FLAT 0  // k_commit: a winner's in-row and hub list walked as one flat range (round 6:
                          // measured slower, R-MAT-24 +1 ms, R-MAT-26 +4.6 ms, profiles/r06/w)
#endif
#ifndef GC_COMMIT_HUB_MIN
#define GC_COMMIT_HUB_MIN 16
#endif
#ifndef GC_VPW_MIN_C
#define GC_VPW_MIN_C 16
#endif


__device__ __forceinline__ void gc_close_body(GDev& g, const GLists& L, DevCtl* c, int mode, int allow_big, int fused) {
    if (threadIdx.x >= GC_WAVE) return;
    const int lane = threadIdx.x;
#if GC_CLOSE_BATCH
    GcCloseCtl kc{};
    if (lane == 0) kc = gc_close_load(c);  // in flight with the counter reads below
#endif
    ull a = 0;  // the commit's slotted winner counts
    if (g.accs)
        for (int k = lane; k < GC_ACC_SLOTS; k += GC_WAVE) a += atomicExch(&g.accs[k], 0ull);
    a = gc_wave_sum(a);
    // the counters the close reads, one lane each, in one memory trip (they were one
    // returning atomic after another: ~1 us each on the round's critical path)
    const int cur = c->cur;
    ull x = 0;
    if (lane == 1) x = gc_aread(&c->accepted);
    else if (lane == 2) x = gc_aread(&c->nx_failcnt);
    else if (lane == 3) x = gc_aread(reinterpret_cast<ull*>(&c->nx_maxmex));
    else if (lane == 4) x = gc_aread(&c->uncolored);
    else if (lane == 5) x = gc_aread(&c->fcnt[mode == GC_CM_ROUND ? cur ^ 1 : cur]);  // the next frontier
    GcClosePre pre;
    pre.accepted = (ull)__shfl((long long)x, 1, GC_WAVE) + a;
    pre.nx_failcnt = (ull)__shfl((long long)x, 2, GC_WAVE);
    pre.nx_maxmex = __shfl((long long)x, 3, GC_WAVE);
    pre.uncolored = (ull)__shfl((long long)x, 4, GC_WAVE);
    pre.fnext = (ull)__shfl((long long)x, 5, GC_WAVE);
#if GC_CLOSE_BATCH
    if (lane == 0) gc_close_batched(g, L, c, mode, allow_big, fused, pre, kc);
#else
    if (lane == 0) gc_close_interleaved(g, L, c, mode, allow_big, fused, pre);
#endif
}

// The whole control block into the host-mapped snapshot slot (one workgroup, every thread
// calls; vector stores).  Words other workgroups of the same launch updated are read with
// atomic RMWs, so no cache holds them back.
__device__ void gc_snap_copy(DevCtl* c, DevCtl* snap) {
    static_assert(sizeof(DevCtl) % 8 == 0, "DevCtl is copied as 8-byte words");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's control-block stores have landed
    __syncthreads();
    ull* src = reinterpret_cast<ull*>(c);
    ull* dst = reinterpret_cast<ull*>(snap);
    for (int i = threadIdx.x; i < (int)(sizeof(DevCtl) / 8); i += blockDim.x) dst[i] = atomicAdd(src + i, 0ull);
    __threadfence_system();
}

// End-of-commit flush that also closes the round (k_commit with tclose): the one returning
// atomic a workgroup already spends on the next frontier's counter also carries an arrival
// ticket in its high bits (count + 2^40), so the workgroup that sees every other arrival
// knows it is last, with every counter atomic of the launch performed before its ticket
// (each wave waits for its own atomics before the workgroup barrier that precedes it).
// Returns true in the last workgroup; *fnext = the next frontier's size.  (Waves whose stage
// filled up flushed earlier with gc_stage_flush, which masks the tickets: GC_COUNT_MASK.)
__device__ __forceinline__ bool gc_stage_flush_ticket(GcStage& s, int* out, ull* out_cnt, ull* fnext) {
    __shared__ int s_cnt[GC_WAVES_PER_BLOCK];
    __shared__ ull s_base, s_fin;
    __shared__ int s_last;
    const int w = threadIdx.x / GC_WAVE;
    gc_wave_sync();
    if (gc_lane() == 0) s_cnt[w] = s.cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int i = 0; i < GC_WAVES_PER_BLOCK; ++i) t += s_cnt[i];
        const ull old = atomicAdd(out_cnt, (1ull << GC_TICKET_SHIFT) | (ull)t);
        s_base = old & GC_COUNT_MASK;
        s_fin = s_base + (ull)t;
        s_last = (old >> GC_TICKET_SHIFT) == (ull)gridDim.x - 1;
    }
    __syncthreads();
    ull base = s_base;
    for (int i = 0; i < w; ++i) base += (ull)s_cnt[i];
    if (gc_stage_fits(s, base)) {
#pragma unroll 1
        for (int i = gc_lane(); i < s.cnt; i += GC_WAVE) out[base + i] = s.buf[i];
    }
    s.cnt = 0;
    *fnext = s_fin;
    return s_last != 0;
}

// The frontier of a big round (F >= n/64, with the host's allow_big) is not appended to:
// it is every claimed uncoloured vertex, rebuilt in vertex order from the claim bitmap by
// k_front_count / k_fsort_scan / k_fsort_write after the commit -- losers are claimed
// already, newly reached vertices get claimed without atomics:
//   push  each winner marks its in-neighbours with plain byte stores (mark[x] = 1), which
//         k_front_count merges into inF;
//   pull  once the dormant set -- uncoloured vertices with no coloured listed neighbour,
//         U - F of them -- is small next to the frontier, the winners' in-edges mostly hit
//         vertices already claimed; the dormant vertices scan their own rows instead
//         (k_pull) and claim themselves.
// Small rounds keep the claim-and-append push.  The next frontier is the same set in
// every case.
__device__ __forceinline__ bool gc_pull_on(const DevCtl* c) {
    const long long F = (long long)c->fcnt[c->cur];
    return 2 * (c->U - F) <= F && !c->pull_off;
}

// Fused commit (k_commit<1>; low-degree graphs, no heavy and no wide proposer possible):
// the wave that stages a vertex for the next frontier also makes its proposal for the
// next round (k_propose's mex, coloring.py:44-54), saving the next round's k_propose
// launch.  Every winner of this round is decided before the commit starts, but another
// wave may not have written its c8 byte yet; under a fused commit a winner keeps its k8
// byte (IN, candidate = its colour), so colour(u) = c8[u] if set, else the candidate of
// an IN k8[u], else none.  (A stale IN byte of an earlier winner never blocks a JP step:
// a proposer's candidate differs from every coloured listed neighbour's colour.)
#ifndef GC_FSLOTS
#define GC_FSLOTS 4
#endif
__device__ __forceinline__ void gc_fused_propose(GDev& g, const int* buf, int cnt, ull* s_mask, long long* s_start,
                                                 long long kbound, long long& lmax, ull& lfail, ull& lsum, ull& lnv) {
    const int lane = gc_lane();
    for (int b = 0; b < cnt; b += GC_WAVE) {  // cnt is wave-uniform
        const int i = b + lane;
        int v = i < cnt ? buf[i] : -1;
#if GC_CHECKS
        if (v >= g.n || v < -1) {
            gc_dbg(g.ctl, 40, v, i, cnt);
            v = -1;
        }
#endif
        const int d = v >= 0 ? g.deg[v] : 0;
        s_mask[lane] = 0;
        s_start[lane] = v >= 0 ? g.rp[v] : 0;
        const int incl = gc_wave_incl_scan(d);
        const int excl = incl - d;
        const int total = __shfl(incl, GC_WAVE - 1, GC_WAVE);
        gc_wave_sync();
        gc_chunk_edges<GC_FSLOTS>(
            g.col, s_start, excl, total,
            [&](int u) {
                const unsigned cb = g.c8[u], kb = g.k8[u];
                if (cb != GC_C8_NONE) return cb;
                if (gc_k8_state(kb) != GC_JP_IN) return 255u;
                const unsigned c6 = gc_k8_cand(kb);
                return c6 == GC_K8_BIG ? (unsigned)g.cand[u] : c6;
            },
            [&](int o, int, unsigned cc) {
                if (cc < 64u) atomicOr(&s_mask[o], 1ull << cc);
            });
        gc_wave_sync();
        if (v >= 0) {
            const int mex = __builtin_ctzll(~s_mask[lane]);  // deg < 64: the mask is never full
            gc_set_cand(g, v, mex);
            lmax = mex > lmax ? mex : lmax;
            if (kbound >= 0 && mex >= kbound) lfail++;
            lsum += (ull)d;
            lnv++;
        }
        gc_wave_sync();
    }
}

// mode GC_CM_ROUND: light = F[cur] (hubs skipped), heavy = the heavy list, output F[cur^1];
// GC_CM_INIT / GC_CM_RESEED: light = seeds[0], heavy = seeds[1], output F[cur].
// nsweeps: sweeps enqueued for this round; undecided vertices left in the last sweep's
// slot mean the host must enqueue more sweeps first (GC_H_SWEEPS, resume after nsweeps).
// tclose (ROUND mode, no big-round rebuild and no k_commit_big after it): the last
// workgroup closes the round itself (k_close's work, see gc_stage_flush_ticket) and, with
// snap, writes the snapshot; an early return on a halt still writes the snapshot.
template <int FUSE>
__global__ void __launch_bounds__(GC_BLOCK) k_commit(GDev g, GLists L, int mode, int nsweeps, int allow_big,
                                                     DevCtl* snap, int tclose) {
    DevCtl* c = g.ctl;
    const bool shard_check = mode == GC_CM_SHARD && nsweeps == GC_SHARD_CHECK;
    if ((mode == GC_CM_ROUND || shard_check) && c->halt) {
        if (snap && blockIdx.x == 0) gc_snap_copy(c, snap);
        return;
    }
    __shared__ int s_stage[GC_WAVES_PER_BLOCK][GC_STAGE_CAP];
    __shared__ ull s_pmask[FUSE ? GC_WAVES_PER_BLOCK : 1][GC_WAVE];
    __shared__ long long s_pstart[FUSE ? GC_WAVES_PER_BLOCK : 1][GC_WAVE];
    __shared__ long long s_start[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_cc[GC_WAVES_PER_BLOCK][GC_WAVE];
#if GC_COMMIT_FLAT
    __shared__ long long s_hs[FUSE ? 1 : GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_din[FUSE ? 1 : GC_WAVES_PER_BLOCK][GC_WAVE];
#endif
    __shared__ ull scratch[2 * GC_WAVES_PER_BLOCK];
    __shared__ int s_acc, s_accc, s_lose;
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    // k_sweep_tail ran before (nsweeps >= 0), else only the first sweep (k_resolve, slot 0) did
    const long long last = mode == GC_CM_ROUND ? (nsweeps < 0 ? 0ll : c->tail_last) : (shard_check ? c->tail_last : nsweeps);
    const int last_slot = (int)(last % 3);
    if ((mode == GC_CM_ROUND || shard_check) &&
        ((c->und_cnt[last_slot] | c->undh_cnt[last_slot]) || (g.hub_w && c->heavy_cnt && c->hub_start > last))) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            c->sweeps_enq = last;
            c->halt = GC_H_SWEEPS;
        }
        if (snap && blockIdx.x == 0) gc_snap_copy(c, snap);
        return;
    }
    const int cur = c->cur;
    const int round = mode == GC_CM_INIT ? 0 : (int)(c->round + 1);
    const bool want_cround = c->want_cround != 0;
    const bool rnd = mode == GC_CM_ROUND || mode == GC_CM_SHARD;
    const int* __restrict__ list = rnd ? L.F[cur] : L.seeds[0];
    const long long cnt = (long long)(rnd ? c->fcnt[cur] : c->seed_cnt[0]);
    const int* hlist = rnd ? L.heavy : L.seeds[1];
    const long long hcnt = (long long)(rnd ? c->heavy_cnt : c->seed_cnt[1]);
    const int skip_heavy = rnd;
    const int nxt = rnd ? cur ^ 1 : cur;
    int* next = L.F[nxt];
    ull* next_cnt = &c->fcnt[nxt];
    const bool big = mode == GC_CM_ROUND && allow_big && gc_big_on(g, c);  // next list: k_front_*
    const bool mark = big && !gc_pull_on(c);                              // else k_pull claims
    GcStage st{s_stage[w], 0, g.list_cap, &g.ctl->loop_err, &g.ctl->halt};
    long long lmaxc = -1;
    ull lacc = 0, lsum = 0;
#if GC_CHECKS
    if (cnt > g.n || hcnt > g.n || (long long)(*next_cnt & GC_COUNT_MASK) > g.n) {
        // this workgroup takes no arrival ticket, so no closing workgroup would write the
        // snapshot: halt the pipeline and write it here (loop_err 3 is in it)
        if (threadIdx.x == 0) {
            gc_dbg(c, 10 + mode, cnt, hcnt, (long long)*next_cnt);
            __hip_atomic_store(&c->halt, GC_H_STALLED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (tclose && snap) gc_snap_copy(c, snap);
        return;
    }
#endif
    // fused: the next round's proposals of the staged vertices (before every flush)
    const long long kbound = c->kbound;
    long long pmax = -1;
    ull pfail = 0, psum = 0, pnv = 0;
    auto propose_staged = [&]() {
        if (FUSE) gc_fused_propose(g, st.buf, st.cnt, s_pmask[FUSE ? w : 0], s_pstart[FUSE ? w : 0], kbound, pmax, pfail,
                                   psum, pnv);
    };
    auto push = [&](bool pred, int val) {
#if GC_CHECKS
        if (pred && (val < 0 || val >= g.n)) {
            gc_dbg(c, 50, val, st.cnt, (long long)*next_cnt);
            pred = false;
        }
#endif
        if (FUSE) {
            const int np = __popcll(__ballot(pred));
            if (np && st.cnt + np > GC_STAGE_CAP) {
                propose_staged();
                gc_stage_flush(st, next, next_cnt);
            }
        }
        gc_stage_push(st, pred, val, next, next_cnt);
    };
    // a winner's in-row [ts, te) strided over the calling threads (a wave, or the workgroup):
    // every in-neighbour marked (big round) or claimed into the next frontier
    auto walk_claims = [&](long long ts, long long te, int t0, int step) {
        for (long long e0 = ts; e0 < te; e0 += step) {
            const long long e = e0 + t0;
            bool claim = false;
            int x = 0;
            if (e < te) {
                x = g.tcol[e];
                if (mark) gc_mark(g, x);
                else claim = gc_claim(g.inF, x);
            }
            push(claim, x);
        }
    };
    // hubs on: each wave takes a run of up to 64 consecutive heavy entries, one per lane, so a
    // whole run's list and state words are loaded in one trip each (round 6, GC_COMMIT_HUB_LANES:
    // a wave per hub walked ~60 hubs one after another in a big round -- two dependent trips
    // each, ~120 trips per wave); its winners' rows are then walked by the whole wave, one
    // winner at a time (in-rows past bigrow are deferred to k_commit_big)
    if (g.hub_w && GC_COMMIT_HUB_LANES) {
        const long long W = (long long)gridDim.x * GC_WAVES_PER_BLOCK;
        const long long wid = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w;
        // (at least GC_COMMIT_HUB_MIN entries a run: fewer waves and workgroups hold losers, and
        // each holding workgroup's flush is an atomic on the next frontier's counter)
        const long long per = std::min<long long>(GC_WAVE, std::max<long long>(GC_COMMIT_HUB_MIN, (hcnt + W - 1) / W));
        for (long long i0 = wid * per; i0 < hcnt; i0 += W * per) {
            const long long i = i0 + lane;
            const int v = (lane < per && i < hcnt) ? hlist[i] : -1;
            const unsigned kv = v >= 0 ? (unsigned)g.k8[v] : 0u;
            const unsigned js = v >= 0 ? gc_k8_state(kv) : (unsigned)GC_JP_UND;
            const bool win = js == GC_JP_IN;
            int cc = 0;
            bool walk = false;
            if (win) {
                const int cb = g.cand[v];
                const long long ts = g.trp[v], te = g.trp[v + 1];
                const long long hn = g.hin_rp[v + 1] - g.hin_rp[v];
                cc = gc_k8_cand(kv) == GC_K8_BIG ? cb : (int)gc_k8_cand(kv);
                const long long tl = te - ts;
                walk = tl + hn <= g.bigrow;
                gc_commit_colour(g, v, cc);
                if (want_cround) g.cround[v] = round;
                lmaxc = cc > lmaxc ? cc : lmaxc;
                lacc++;
                lsum += (ull)tl;
            }
            gc_wave_append(win && !walk, v, L.bigw, &c->bigw_cnt);  // the whole grid walks it
            push(js == GC_JP_OUT && !big, v);                       // losers stay
            for (ull wm = __ballot(walk); wm; wm &= wm - 1) {
                const int l = __ffsll((long long)wm) - 1;
                const int wv = __shfl(v, l, GC_WAVE);
                const int wc = __shfl(cc, l, GC_WAVE);
                gc_hub_mark_row(g, wv, wc, lane, GC_WAVE);  // gc_hubs.hip
                if (mark || !big) walk_claims(g.trp[wv], g.trp[wv + 1], lane, GC_WAVE);
            }
        }
    } else if (g.hub_w) {  // a wave per hub (round 5)
        for (long long i = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w; i < hcnt;
             i += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
            const int v = hlist[i];
            const unsigned kv = g.k8[v];
            const unsigned js = gc_k8_state(kv);
            bool walk = js == GC_JP_IN;
            int cc = 0;
            if (walk) {
                cc = gc_k8_cand(kv) == GC_K8_BIG ? g.cand[v] : (int)gc_k8_cand(kv);
                const long long tl = g.trp[v + 1] - g.trp[v];
                walk = tl + (g.hin_rp[v + 1] - g.hin_rp[v]) <= g.bigrow;
                if (lane == 0) {
                    gc_commit_colour(g, v, cc);
                    if (want_cround) g.cround[v] = round;
                    lmaxc = cc > lmaxc ? cc : lmaxc;
                    lacc++;
                    lsum += (ull)tl;
                    if (!walk) L.bigw[atomicAdd(&c->bigw_cnt, 1ull)] = v;  // the whole grid walks it
                }
            }
            push(lane == 0 && js == GC_JP_OUT && !big, v);  // losers stay
            if (walk) {
                gc_hub_mark_row(g, v, cc, lane, GC_WAVE);  // gc_hubs.hip
                if (mark || !big) {
                    const long long ts = g.trp[v], te = g.trp[v + 1];
                    walk_claims(ts, te, lane, GC_WAVE);
                }
            }
        }
    }
    // hubs off: a workgroup per heavy vertex
    for (long long i = blockIdx.x; i < (g.hub_w ? 0ll : hcnt); i += gridDim.x) {
        const int v = hlist[i];
        if (threadIdx.x == 0) {
            const unsigned kv = g.k8[v];
            const unsigned js = gc_k8_state(kv);
            s_acc = js == GC_JP_IN;
            if (js == GC_JP_IN) {
                const int cc = gc_k8_cand(kv) == GC_K8_BIG ? g.cand[v] : (int)gc_k8_cand(kv);
                gc_commit_colour(g, v, cc);
                s_accc = cc;
                if (want_cround) g.cround[v] = round;
                lmaxc = cc > lmaxc ? cc : lmaxc;
                lacc++;
                const long long rows = (g.trp[v + 1] - g.trp[v]) + (g.hbits_w ? g.hin_rp[v + 1] - g.hin_rp[v] : 0);
                lsum += (ull)(g.trp[v + 1] - g.trp[v]);
                if (rows > g.bigrow) {  // the whole grid walks it (k_commit_big)
                    L.bigw[atomicAdd(&c->bigw_cnt, 1ull)] = v;
                    s_acc = 0;
                }
            }
            s_lose = js == GC_JP_OUT && !big;
        }
        __syncthreads();
        if (w == 0) push(lane == 0 && s_lose, v);  // losers stay
        if (s_acc && g.hbits_w) gc_hub_mark_row(g, v, s_accc, threadIdx.x, blockDim.x);  // gc_hubs.hip
        if (s_acc && (mark || !big)) walk_claims(g.trp[v], g.trp[v + 1], threadIdx.x, blockDim.x);
        __syncthreads();
    }
    // light vertices: wave chunks (at least GC_VPW_MIN_C vertices each, round 6: as above)
    int vpw = gc_vpw(cnt, (long long)gridDim.x * GC_WAVES_PER_BLOCK);
    if (!FUSE && vpw < GC_VPW_MIN_C) vpw = GC_VPW_MIN_C;  // (the fused commit's graphs have no hub list)
    const long long nch = gc_nchunks(cnt, vpw);
    for (long long ch = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w; ch < nch;
         ch += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
        const long long idx = ch * vpw + lane;
        int v = (lane < vpw && idx < cnt) ? list[idx] : -1;
#if GC_CHECKS
        if (v >= g.n || v < -1) {
            gc_dbg(c, 20, v, idx, cnt);
            v = -1;
        }
#endif
        // the vertex's words are loaded together (its in-row bounds before knowing it won:
        // one memory trip instead of two); fused: no heavy vertex, so no degree needed
        const int d = (v >= 0 && !FUSE) ? g.deg[v] : 0;
        const unsigned kv0 = v >= 0 ? (unsigned)g.k8[v] : 0u;
#if GC_HOIST_HIN
        const int cb0 = v >= 0 ? g.cand[v] : 0;
        const long long hs0 = (v >= 0 && g.hbits_w) ? g.hin_rp[v] : 0;
        const long long he0 = (v >= 0 && g.hbits_w) ? g.hin_rp[v + 1] : 0;
#endif
#if GC_PREFETCH_ROW
        const long long ts0 = v >= 0 ? g.trp[v] : 0, te0 = v >= 0 ? g.trp[v + 1] : 0;
#else
        const long long ts0 = (v >= 0 && gc_k8_state(kv0) == GC_JP_IN) ? g.trp[v] : 0;
        const long long te0 = (v >= 0 && gc_k8_state(kv0) == GC_JP_IN) ? g.trp[v + 1] : 0;
#endif
        const bool skip = v < 0 || (skip_heavy && d > g.heavy_t);
        const unsigned kv = skip ? 0u : kv0;
        const unsigned js = skip ? (unsigned)GC_JP_UND : gc_k8_state(kv);
        const bool acc = js == GC_JP_IN;
        int din = 0, cc = 0;
        long long tstart = 0;
        if (acc) {
#if GC_HOIST_HIN
            cc = gc_k8_cand(kv) == GC_K8_BIG ? cb0 : (int)gc_k8_cand(kv);
#else
            cc = gc_k8_cand(kv) == GC_K8_BIG ? g.cand[v] : (int)gc_k8_cand(kv);
#endif
            if (FUSE) gc_commit_colour_keep(g, v, cc);
            else gc_commit_colour(g, v, cc);
            if (want_cround) g.cround[v] = round;
            lmaxc = cc > lmaxc ? cc : lmaxc;
            lacc++;
            tstart = ts0;
            din = (int)(te0 - tstart);
            lsum += (ull)din;
            if (big && !mark) din = 0;
        }
        // losers stay in the frontier (they still have a coloured neighbour)
        push(js == GC_JP_OUT && !big, v);
#if GC_COMMIT_FLAT
        if (!FUSE && g.hbits_w) {
            // the winners' in-rows (claims / marks) and hub lists (colour pushes) as ONE flat
            // range of the wave (round 6): the two walks' loads in flight together instead of
            // one walk after the other
            long long hs = 0;
            int dh = 0;
            if (acc) {
                hs = g.hin_rp[v];
                dh = (int)(g.hin_rp[v + 1] - hs);
            }
            s_start[w][lane] = tstart;
            s_hs[w][lane] = hs;
            s_din[w][lane] = din;
            s_cc[w][lane] = cc;
            const int len = din + dh;
            const int fincl = gc_wave_incl_scan(len);
            const int fexcl = fincl - len;
            const int ftotal = __shfl(fincl, GC_WAVE - 1, GC_WAVE);
            gc_wave_sync();
            for (int base = 0; base < ftotal; base += GC_CSLOTS * GC_WAVE) {
                int x[GC_CSLOTS], hc[GC_CSLOTS];
                bool ok[GC_CSLOTS], hub[GC_CSLOTS], claim[GC_CSLOTS];
#pragma unroll
                for (int k = 0; k < GC_CSLOTS; ++k) {
                    const int e = base + k * GC_WAVE + lane;
                    const int o = gc_owner(fexcl, e);
                    const int off = e - __shfl(fexcl, o, GC_WAVE);
                    ok[k] = e < ftotal;
                    const int dno = s_din[w][o];
                    hub[k] = ok[k] && off >= dno;
                    hc[k] = s_cc[w][o];
                    x[k] = !ok[k] ? 0 : (hub[k] ? g.hin_col[s_hs[w][o] + (off - dno)] : g.tcol[s_start[w][o] + off]);
                }
#pragma unroll
                for (int k = 0; k < GC_CSLOTS; ++k) {
                    claim[k] = false;
                    if (!ok[k]) continue;
                    if (hub[k]) gc_hub_mark(g, x[k], hc[k]);
                    else if (mark) gc_mark(g, x[k]);
                    else claim[k] = gc_claim(g.inF, x[k]);
                }
#pragma unroll
                for (int k = 0; k < GC_CSLOTS; ++k) push(claim[k], x[k]);
            }
            gc_wave_sync();
            continue;
        }
#endif
        s_start[w][lane] = tstart;
        const int incl = gc_wave_incl_scan(din);
        const int excl = incl - din;
        const int total = __shfl(incl, GC_WAVE - 1, GC_WAVE);
        gc_wave_sync();
        // GC_CSLOTS 64-edge groups per step: their tcol loads, then their claims, in flight
        // together (GC_CLAIM_DIRECT=1, fused: one atomic per claim without the check-load;
        // measured slower on meshes: neighbours share claim words)
        for (int base = 0; base < total; base += GC_CSLOTS * GC_WAVE) {
            int x[GC_CSLOTS];
            bool ok[GC_CSLOTS], claim[GC_CSLOTS];
#pragma unroll
            for (int k = 0; k < GC_CSLOTS; ++k) {
                const int e = base + k * GC_WAVE + lane;
                const int o = gc_owner(excl, e);
                const int eo = __shfl(excl, o, GC_WAVE);
                ok[k] = e < total;
                x[k] = ok[k] ? g.tcol[s_start[w][o] + (e - eo)] : 0;
#if GC_CHECKS
                if (ok[k] && (x[k] < 0 || x[k] >= g.n)) {
                    gc_dbg(c, 30, x[k], s_start[w][o] + (e - eo), e);
                    ok[k] = false;
                }
#endif
            }
#pragma unroll
            for (int k = 0; k < GC_CSLOTS; ++k) {
                claim[k] = false;
                if (ok[k]) {
                    if (mark) gc_mark(g, x[k]);
                    else if (FUSE && g.claim_direct) claim[k] = gc_claim_direct(g.inF, x[k]);
                    else claim[k] = gc_claim(g.inF, x[k]);
                }
            }
#pragma unroll
            for (int k = 0; k < GC_CSLOTS; ++k) push(claim[k], x[k]);
        }
        if (g.hbits_w) {  // push the winners' colours into the hubs that list them (gc_hubs.hip)
            int dh = 0;
            if (acc) {
#if GC_HOIST_HIN
                tstart = hs0;
                dh = (int)(he0 - hs0);
#else
                tstart = g.hin_rp[v];
                dh = (int)(g.hin_rp[v + 1] - tstart);
#endif
            }
            gc_wave_sync();
            s_start[w][lane] = tstart;
            s_cc[w][lane] = cc;
            const int hincl = gc_wave_incl_scan(dh);
            const int hexcl = hincl - dh;
            const int htotal = __shfl(hincl, GC_WAVE - 1, GC_WAVE);
            gc_wave_sync();
            gc_hub_mark_flat(g, htotal, [&](int e, int* x, int* c) {
                const int o = gc_owner(hexcl, e);
                const int eo = __shfl(hexcl, o, GC_WAVE);
                *x = e < htotal ? g.hin_col[s_start[w][o] + (e - eo)] : -1;
                *c = e < htotal ? s_cc[w][o] : 0;
            });
        }
        gc_wave_sync();
    }
    propose_staged();
    if (!tclose) gc_stage_flush_block(st, next, next_cnt);
    __syncthreads();
    gc_block_max(&c->maxcolor, lmaxc, (long long*)scratch);
    if (FUSE) {
        gc_block_max(&c->nx_maxmex, pmax, (long long*)scratch);
        gc_block_add(&c->nx_failcnt, pfail, scratch);
        gc_stat_add(g, GC_K_PROPOSE, psum, pnv, scratch);
    }
    if (g.accs) {  // slotted (k_close sums them): 1024 workgroups on one counter cost ~10 us
        const ull wacc = gc_wave_sum(lacc);
        if (gc_lane() == 0 && wacc) atomicAdd(&g.accs[(blockIdx.x * GC_WAVES_PER_BLOCK + w) % GC_ACC_SLOTS], wacc);
    } else {
        gc_block_add(&c->accepted, lacc, scratch);
    }
    gc_stat_add(g, GC_K_COMMIT, lsum, lacc, scratch);
    if (tclose) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's counter atomics are performed
        ull fnext = 0;
        if (gc_stage_flush_ticket(st, next, next_cnt, &fnext)) {  // the last workgroup closes the round
            if (threadIdx.x == 0) gc_st(next_cnt, fnext);            // without the tickets
            __syncthreads();
            gc_close_body(g, L, c, mode, 0, FUSE);
            if (snap) gc_snap_copy(c, snap);
        }
    }
}

// Winners whose in-rows exceed bigrow (GC_BIGROW), deferred by k_commit: the grid walks the
// concatenation of every such winner's rows (colour pushes into the hubs listing the
// winner, then the frontier claims / marks of its in-neighbours) as one flat index space,
// 256 winners per tile (their row offsets prefix-summed in LDS, owner by binary search).
// Walking the winners one after another cost ~5 dependent memory round trips per winner
// on every workgroup: 1.8 ms for the ~400 hub winners of an R-MAT-26 round.
// tclose (round 6, GC_CB_CLOSE; the one-GPU engine's small rounds): the last workgroup closes the
// round (k_close's work and the snapshot), found by arrival tickets counted per dispatch residue
// (blockIdx % 8, ~1/8 of the workgroups on each of eight counters, then eight arrivals on a top
// counter) -- round 4's single counter for 1024 workgroups cost more than the k_close it saved
__device__ __forceinline__ bool gc_cb_ticket(ull* tick) {
    __shared__ int s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's counter atomics are performed
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned sh = blockIdx.x & 7u;
        const ull nsh = (ull)((gridDim.x - sh + 7u) / 8u);  // workgroups of this residue
        const ull ntop = gridDim.x < 8u ? (ull)gridDim.x : 8ull;
        int last = 0;
        if (atomicAdd(&tick[8 * sh], 1ull) + 1ull == nsh) {
            gc_st(&tick[8 * sh], 0ull);  // every arrival of this residue is in
            if (atomicAdd(&tick[64], 1ull) + 1ull == ntop) {
                gc_st(&tick[64], 0ull);
                last = 1;
            }
        }
        s_last = last;
    }
    __syncthreads();
    return s_last != 0;
}
__global__ void __launch_bounds__(GC_BLOCK) k_commit_big(GDev g, GLists L, int mode, int allow_big, DevCtl* snap,
                                                         int tclose) {
    DevCtl* c = g.ctl;
    if (mode == GC_CM_ROUND && c->halt) {
        if (tclose && snap && blockIdx.x == 0) gc_snap_copy(c, snap);
        return;
    }
    const long long nb = (long long)c->bigw_cnt;
    if (nb == 0) {
        if (tclose && gc_cb_ticket(g.accs + GC_ACC_SLOTS)) {
            gc_close_body(g, L, c, mode, 0, 0);
            if (snap) gc_snap_copy(c, snap);
        }
        return;
    }
    __shared__ int s_stage[GC_WAVES_PER_BLOCK][GC_STAGE_CAP];
    __shared__ long long s_off[GC_BLOCK + 1];  // exclusive prefix of the tile's per-winner work
    __shared__ long long s_hs[GC_BLOCK], s_ts[GC_BLOCK];
    __shared__ int s_hl[GC_BLOCK], s_cc[GC_BLOCK];
    __shared__ long long s_wsum[GC_WAVES_PER_BLOCK];
    const int t = threadIdx.x;
    const int lane = gc_lane();
    const int w = t / GC_WAVE;
    const bool rnd = mode == GC_CM_ROUND || mode == GC_CM_SHARD;
    const int cur = c->cur;
    const int nxt = rnd ? cur ^ 1 : cur;
    int* next = L.F[nxt];
    ull* next_cnt = &c->fcnt[nxt];
    const bool big = mode == GC_CM_ROUND && allow_big && gc_big_on(g, c);
    const bool mark = big && !gc_pull_on(c);
    const bool walk_t = mark || !big;
    GcStage st{s_stage[w], 0, g.list_cap, &g.ctl->loop_err, &g.ctl->halt};
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long j0 = 0; j0 < nb; j0 += GC_BLOCK) {
        const int tn = (int)(nb - j0 < GC_BLOCK ? nb - j0 : GC_BLOCK);
        long long len = 0;
        if (t < tn) {
            const int v = L.bigw[j0 + t];
            int hl = 0;
            if (g.hbits_w) {
                s_hs[t] = g.hin_rp[v];
                hl = (int)(g.hin_rp[v + 1] - s_hs[t]);
                s_cc[t] = gc_colour(g, v);
            }
            s_hl[t] = hl;
            s_ts[t] = g.trp[v];
            len = hl + (walk_t ? g.trp[v + 1] - s_ts[t] : 0ll);
        }
        // workgroup inclusive scan of len
        long long x = len;
#pragma unroll
        for (int o = 1; o < GC_WAVE; o <<= 1) {
            const long long y = __shfl_up(x, o, GC_WAVE);
            if (lane >= o) x += y;
        }
        if (lane == GC_WAVE - 1) s_wsum[w] = x;
        __syncthreads();
        for (int k = 0; k < w; ++k) x += s_wsum[k];
        s_off[t + 1] = x;
        if (t == 0) s_off[0] = 0;
        __syncthreads();
        const long long total = s_off[tn];
#if GC_CB_UNR > 1
        // GC_CB_UNR entries a thread per step, their loads in flight together (round 6: one
        // entry a step paid its dependent trips -- entry, claim word, atomic -- per entry)
        for (long long f0 = (long long)blockIdx.x * blockDim.x * GC_CB_UNR; f0 < total; f0 += stride * GC_CB_UNR) {
            int ent[GC_CB_UNR], kk[GC_CB_UNR];
            bool hub[GC_CB_UNR], ok[GC_CB_UNR];
#pragma unroll
            for (int u = 0; u < GC_CB_UNR; ++u) {
                const long long f = f0 + (long long)u * blockDim.x + t;
                ok[u] = f < total;
                int k = 0;  // max k < tn with s_off[k] <= f
                if (ok[u]) {
#pragma unroll
                    for (int step = GC_BLOCK / 2; step > 0; step >>= 1)
                        if (k + step < tn && s_off[k + step] <= f) k += step;
                }
                kk[u] = k;
                const long long off = ok[u] ? f - s_off[k] : 0;
                hub[u] = ok[u] && off < s_hl[k];
                ent[u] = !ok[u] ? 0 : (hub[u] ? g.hin_col[s_hs[k] + off] : g.tcol[s_ts[k] + (off - s_hl[k])]);
            }
            // the check words first (claim word, or the hub's bitmap word), then the writes
            unsigned* wp[GC_CB_UNR];
            unsigned bit[GC_CB_UNR], wd[GC_CB_UNR];
#pragma unroll
            for (int u = 0; u < GC_CB_UNR; ++u) {
                wp[u] = nullptr;
                bit[u] = 0u;
                if (ok[u]) {
                    if (hub[u]) {
                        const int cc = s_cc[kk[u]];
                        if (cc < 32 * g.hbits_w) {
                            wp[u] = gc_hbw(g, ent[u], cc >> 5);
                            bit[u] = 1u << (cc & 31);
                        }
                    } else {
                        wp[u] = g.inF + (ent[u] >> 5);
                        bit[u] = 1u << (ent[u] & 31);
                    }
                }
                wd[u] = wp[u] ? *wp[u] : 0xFFFFFFFFu;
            }
            bool claim[GC_CB_UNR];
#pragma unroll
            for (int u = 0; u < GC_CB_UNR; ++u) {
                claim[u] = false;
                if (!ok[u]) continue;
                if (hub[u]) {
                    if (g.hseen && !g.hseen[ent[u]]) g.hseen[ent[u]] = 1;  // (gc_hub_mark)
                    if (wp[u] && !(wd[u] & bit[u])) atomicOr(wp[u], bit[u]);
                } else if (!(wd[u] & bit[u])) {
                    if (mark) g.mark[ent[u]] = 1;  // (gc_mark: its claim bit is clear)
                    else claim[u] = !(atomicOr(wp[u], bit[u]) & bit[u]);
                }
            }
#pragma unroll
            for (int u = 0; u < GC_CB_UNR; ++u) gc_stage_push(st, claim[u], ent[u], next, next_cnt);
        }
#else
        for (long long f0 = (long long)blockIdx.x * blockDim.x; f0 < total; f0 += stride) {
            const long long f = f0 + t;
            bool claim = false;
            int xv = 0;
            if (f < total) {
                int k = 0;  // max k < tn with s_off[k] <= f
#pragma unroll
                for (int step = GC_BLOCK / 2; step > 0; step >>= 1)
                    if (k + step < tn && s_off[k + step] <= f) k += step;
                const long long off = f - s_off[k];
                if (off < s_hl[k]) {
                    gc_hub_mark(g, g.hin_col[s_hs[k] + off], s_cc[k]);
                } else {
                    xv = g.tcol[s_ts[k] + (off - s_hl[k])];
                    if (mark) gc_mark(g, xv);
                    else claim = gc_claim(g.inF, xv);
                }
            }
            gc_stage_push(st, claim, xv, next, next_cnt);
        }
#endif
        __syncthreads();  // the tile's LDS is rewritten next
    }
    gc_stage_flush_block(st, next, next_cnt);
    if (tclose && gc_cb_ticket(g.accs + GC_ACC_SLOTS)) {
        gc_close_body(g, L, c, mode, 0, 0);
        if (snap) gc_snap_copy(c, snap);
    }
}

// Pull half of a big round (see gc_big_on): every dormant vertex -- unclaimed in inF, hence
// uncoloured with no coloured listed neighbour before this round -- scans its own row for
// a neighbour coloured now and claims itself.  A wave owns 64 consecutive vertices, i.e.
// two whole inF words, so the claims are plain stores.
__global__ void __launch_bounds__(GC_BLOCK) k_pull(GDev g, int allow_big) {
    DevCtl* c = g.ctl;
    if (!gc_front_on(g, c, allow_big) || !gc_pull_on(c)) return;
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    const long long n = g.n;
    const long long steps = (n + GC_WAVE - 1) / GC_WAVE;
    for (long long sidx = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w; sidx < steps;
         sidx += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
        const long long v = sidx * GC_WAVE + lane;
        const unsigned word = v < n ? g.inF[v >> 5] : 0xFFFFFFFFu;
        const bool dorm = v < n && !((word >> (v & 31)) & 1u);
        if (!__ballot(dorm)) continue;
        bool hit = false;
        if (dorm && g.c8[v] == GC_C8_NONE) {
            const long long ee = g.rp[v + 1];
            for (long long e = g.rp[v]; e < ee && !hit; ++e) hit = g.c8[g.col[e]] != GC_C8_NONE;
        }
        const ull m = __ballot(hit);
        if (lane == 0 && (unsigned)m) g.inF[v >> 5] = word | (unsigned)m;
        if (lane == 32 && (unsigned)(m >> 32)) g.inF[v >> 5] = word | (unsigned)(m >> 32);
    }
}

// Next frontier of a big round, pass 1: merge this word's marks into the claim bitmap
// (clearing them) and count its claimed uncoloured vertices per workgroup.  Passes 2/3 are
// k_fsort_scan / k_fsort_write with build = 1 (next list slot, count from the scan).
__global__ void __launch_bounds__(GC_BLOCK) k_front_count(GDev g, unsigned* bsum) {
    DevCtl* c = g.ctl;
    if (!gc_front_on(g, c, 1)) return;
    __shared__ ull scratch[2 * GC_WAVES_PER_BLOCK];
    const long long words = ((long long)g.n + 31) / 32;
    const long long w = (long long)blockIdx.x * GC_BLOCK + threadIdx.x;
    ull cnt = 0;
    if (w < words) {
        const long long v0 = w * 32;
        unsigned mk = 0u;
        if (v0 + 32 <= (long long)g.n) {
            uint4* p = reinterpret_cast<uint4*>(g.mark + v0);
            const uint4 a = p[0], b = p[1];
            const unsigned x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
            for (int k = 0; k < 8; ++k)  // mark bytes are 0 or 1
                mk |= ((x[k] & 1u) | ((x[k] >> 7) & 2u) | ((x[k] >> 14) & 4u) | ((x[k] >> 21) & 8u)) << (4 * k);
            if (mk) p[0] = p[1] = make_uint4(0u, 0u, 0u, 0u);
        } else {
            for (int k = 0; k < 32 && v0 + k < (long long)g.n; ++k)
                if (g.mark[v0 + k]) {
                    mk |= 1u << k;
                    g.mark[v0 + k] = 0;
                }
        }
        if (mk) g.inF[w] |= mk;  // this thread owns the word
        cnt = (ull)__popc(gc_front_word(g, w));
    }
    cnt = gc_wave_sum(cnt);
    if (gc_lane() == 0) scratch[threadIdx.x / GC_WAVE] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        ull t = 0;
        for (int i = 0; i < GC_WAVES_PER_BLOCK; ++i) t += scratch[i];
        bsum[blockIdx.x] = (unsigned)t;
    }
}

// Closes the round (or the INIT / RESEED seeding) after its commit: one thread, so every
// counter the commit's workgroups updated is visible across the launch boundary.

// snap (host-mapped, or null): afterwards the whole control block is copied there, halted or
// not, with vector stores; the host reads it once the batch's event has completed.
__global__ void k_close(GDev g, GLists L, int mode, int allow_big, int fused, DevCtl* snap) {
    DevCtl* c = g.ctl;
    if (!(mode == GC_CM_ROUND && c->halt)) gc_close_body(g, L, c, mode, allow_big, fused);
    if (snap) gc_snap_copy(c, snap);
}

// ------------------------------------------------------------------------------------
// Sharded rounds (gc_shard.hip): a rank runs the round kernels on its own
// frontier; at the three grid-wide seams it publishes (vertex << 32 | value) deltas of
// its vertices and applies everyone else's.
// ------------------------------------------------------------------------------------
// propose seam: (v, candidate) for every frontier entry of this rank
__global__ void __launch_bounds__(GC_BLOCK) k_delta_cand(GDev g, GLists L) {
    const DevCtl* c = g.ctl;
    if (c->halt) return;
    const int cur = c->cur;
    const long long cnt = (long long)c->fcnt[cur];
    const int* list = L.F[cur];
    if (g.hub_repl) {  // every rank proposes every hub itself: the lights' deltas, compacted
        const long long steps = (cnt + GC_WAVE - 1) / GC_WAVE;
        for (long long sidx = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / GC_WAVE; sidx < steps;
             sidx += (long long)gridDim.x * (blockDim.x / GC_WAVE)) {
            const long long i = sidx * GC_WAVE + gc_lane();
            const int v = i < cnt ? list[i] : -1;
            const bool send = v >= 0 && g.hid[v] < 0;
            const unsigned k = send ? g.k8[v] : 0u;
            const long long dv = send ? gc_delta(v, gc_k8_cand(k) == GC_K8_BIG ? g.cand[v] : (int)gc_k8_cand(k)) : 0ll;
            gc_wave_append64(send, dv, L.delta, const_cast<ull*>(&c->dcnt));
        }
        return;
    }
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += (long long)gridDim.x * blockDim.x) {
        const int v = list[i];
        const unsigned k = g.k8[v];
        L.delta[i] = gc_delta(v, gc_k8_cand(k) == GC_K8_BIG ? g.cand[v] : (int)gc_k8_cand(k));
    }
}

// Apply received deltas to the vertices this rank does not own ([lo, hi) already hold
// them).  Entries with v < 0 are padding (and the exchange headers, gcolor_amd/shard.py).
// rwin != null: IN states -- other ranks' winners of the round -- are also listed there, so
// the round's end colours them from the list instead of scanning every proposal byte.
// hdr_stride > 0 (a fused propose seam, shard.py): recv is every rank's send buffer of
// hdr_stride words (GC_SEAM_HDR header words + inline deltas); if some rank's finish halted
// (word 4 < 0) or its deltas did not fit inline (word 3 > hdr_stride - GC_SEAM_HDR), nothing
// is applied and the shard halts with GC_H_SEAM (the host takes the unfused path).
__device__ __forceinline__ int gc_hdr_value(long long w) { return (int)(unsigned)(w & 0xFFFFFFFFll); }
__global__ void __launch_bounds__(GC_BLOCK) k_apply(GDev g, int kind, const long long* recv, long long count,
                                                    long long lo, long long hi, int round, int* rwin,
                                                    long long hdr_stride) {
    if (g.ctl->halt) return;
    if (hdr_stride > 0) {
        bool bad = false;
        for (long long p = 0; p * hdr_stride < count; ++p) {
            const long long* h = recv + p * hdr_stride;
            bad |= gc_hdr_value(h[4]) < 0 || (long long)gc_hdr_value(h[3]) > hdr_stride - GC_SEAM_HDR;
        }
        if (bad) {
            if (blockIdx.x == 0 && threadIdx.x == 0) g.ctl->halt = GC_H_SEAM;
            return;
        }
    }
    const bool want_cround = g.ctl->want_cround != 0;
    const int lane = gc_lane();
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i - lane < count; i += stride) {
        const long long e = i < count ? recv[i] : -1ll;
        const int v = (int)(e >> 32);
        const bool act = !(v < 0 || (v >= lo && v < hi));
        const int val = (int)(unsigned)(e & 0xFFFFFFFFll);
        if (act) {
            if (kind == GC_KIND_CAND) {
                const unsigned c6 = gc_c6_of(val);
                if (c6 == GC_K8_BIG) g.cand[v] = val;
                g.k8[v] = gc_k8(c6, GC_JP_UND);
            } else if (kind == GC_KIND_STATE) {
                const unsigned kv = g.k8[v];
                g.k8[v] = (unsigned char)((kv & ~3u) | (unsigned)val);
                if (g.hub_repl && g.hub_w && val == GC_JP_IN && g.hid[v] < 0) {
                    // another rank's light winner flags the hubs that list it and propose its
                    // colour, as a local one does in its sweep (gc_jp_sweep)
                    const int cv = gc_k8_cand(kv) == GC_K8_BIG ? g.cand[v] : (int)gc_k8_cand(kv);
                    for (long long q = g.hin_rp[v]; q < g.hin_rp[v + 1]; ++q) {
                        const int hx = g.hin_col[q];
                        if ((g.hk[hx] >> 2) == (unsigned)cv && !g.hkill[hx]) g.hkill[hx] = 1u;
                    }
                }
            } else {
                gc_commit_colour(g, v, val);
                if (want_cround) g.cround[v] = round;
                atomicMax(&g.ctl->maxcolor, (long long)val);
            }
        }
        if (rwin) gc_wave_append(act && kind == GC_KIND_STATE && val == GC_JP_IN, v, rwin, &g.ctl->rwin_cnt);
    }
}

// End of a sharded round, every delta seam: the other ranks' winners arrived as IN state
// deltas and sit in rwin; each is coloured here too and pushes into this rank's
// in-neighbours (owned targets only), O(winners) instead of k_shard_scan_commit's O(n).
__global__ void __launch_bounds__(GC_BLOCK) k_shard_list_commit(GDev g, GLists L, const int* rwin, int* big) {
    DevCtl* c = g.ctl;
    if (c->halt) return;  // the hub JP did not converge (GC_SHARD_CHECK): the host adds sweeps
    __shared__ int s_stage[GC_WAVES_PER_BLOCK][GC_STAGE_CAP];
    __shared__ long long s_start[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_cc[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ ull scratch[2 * GC_WAVES_PER_BLOCK];
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    const int nxt = c->cur ^ 1;
    int* next = L.F[nxt];
    ull* next_cnt = &c->fcnt[nxt];
    const int round = (int)(c->round + 1);
    const bool want_cround = c->want_cround != 0;
    GcStage st{s_stage[w], 0, g.list_cap, &g.ctl->loop_err, &g.ctl->halt};
    long long lmaxc = -1;
    ull lacc = 0;
    const long long cnt = (long long)c->rwin_cnt;
    for (long long ch = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w; ch * GC_WAVE < cnt;
         ch += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
        const long long idx = ch * GC_WAVE + lane;
        const int v = idx < cnt ? rwin[idx] : -1;
        long long tstart = 0;
        int din = 0, cc = 0;
        if (v >= 0) {
            const unsigned b = g.k8[v];
            cc = gc_k8_cand(b) == GC_K8_BIG ? g.cand[v] : (int)gc_k8_cand(b);
            gc_commit_colour(g, v, cc);
            if (want_cround) g.cround[v] = round;
            lmaxc = cc > lmaxc ? cc : lmaxc;
            lacc++;
            tstart = g.trp[v];
            din = (int)(g.trp[v + 1] - tstart);
        }
        s_start[w][lane] = tstart;
        const int incl = gc_wave_incl_scan(din);
        const int excl = incl - din;
        const int total = __shfl(incl, GC_WAVE - 1, GC_WAVE);
        gc_wave_sync();
        for (int base = 0; base < total; base += GC_WAVE) {
            const int e = base + lane;
            const int o = gc_owner(excl, e);
            const int eo = __shfl(excl, o, GC_WAVE);
            bool claim = false;
            int x = 0;
            if (e < total) {
                x = g.tcol[s_start[w][o] + (e - eo)];
                claim = gc_claim(g.inF, x);
            }
            gc_stage_push(st, claim, x, next, next_cnt);
        }
        gc_wave_sync();
        // and into this rank's replica of the hub bitmaps (gc_hubs.hip)
        if (g.hbits_w) gc_hub_push_wave(g, v >= 0, v, cc, s_start[w], s_cc[w], big, &c->list_cnt);
    }
    gc_stage_flush_block(st, next, next_cnt);
    __syncthreads();
    gc_block_max(&c->maxcolor, lmaxc, (long long*)scratch);
    gc_block_add(&c->accepted, lacc, scratch);
}

// End of a sharded round, after the last sweep seam: every rank holds every proposer's
// final JP state, so the winners of the OTHER ranks are read off the replicated proposal
// bytes (state IN, a candidate) instead of being exchanged: each is coloured here too
// and pushes into this rank's in-neighbours (trp/tcol is the rank-local in-neighbour CSR:
// owned targets only).  The rank's own winners went through k_commit (GC_CM_SHARD).
// One 4-byte word of k8 per lane, 256 vertices per wave step.
__global__ void __launch_bounds__(GC_BLOCK) k_shard_scan_commit(GDev g, GLists L, long long lo, long long hi, int* big) {
    DevCtl* c = g.ctl;
    if (c->halt) return;
    __shared__ int s_stage[GC_WAVES_PER_BLOCK][GC_STAGE_CAP];
    __shared__ long long s_start[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_cc[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ ull scratch[2 * GC_WAVES_PER_BLOCK];
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    const int nxt = c->cur ^ 1;
    int* next = L.F[nxt];
    ull* next_cnt = &c->fcnt[nxt];
    const int round = (int)(c->round + 1);
    const bool want_cround = c->want_cround != 0;
    GcStage st{s_stage[w], 0, g.list_cap, &g.ctl->loop_err, &g.ctl->halt};
    long long lmaxc = -1;
    ull lacc = 0;
    const long long n = g.n;
    const long long steps = (n + 4 * GC_WAVE - 1) / (4 * GC_WAVE);
    for (long long sidx = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w; sidx < steps;
         sidx += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
        const long long v0 = sidx * 4 * GC_WAVE + 4 * lane;
        // skip steps inside the owned range (their winners were committed by k_commit)
        if (sidx * 4 * GC_WAVE >= lo && (sidx + 1) * 4 * GC_WAVE <= hi) continue;
        unsigned word = 0xFCFCFCFCu;  // (NONE, UND) x 4
        if (v0 + 3 < n) {
            word = *reinterpret_cast<const unsigned*>(g.k8 + v0);
        } else {
            for (int k = 0; k < 4; ++k)
                if (v0 + k < n) word = (word & ~(0xFFu << (8 * k))) | ((unsigned)g.k8[v0 + k] << (8 * k));
        }
        for (int k = 0; k < 4; ++k) {
            const long long v = v0 + k;
            const unsigned b = (word >> (8 * k)) & 0xFFu;
            const bool win = v < n && (v < lo || v >= hi) && gc_k8_state(b) == GC_JP_IN && gc_k8_cand(b) != GC_K8_NONE &&
                             !(g.hub_repl && g.hid[v] >= 0);  // replicated hubs: committed by k_commit
            if (!__ballot(win)) continue;
            long long tstart = 0;
            int din = 0, cc = 0;
            if (win) {
                cc = gc_k8_cand(b) == GC_K8_BIG ? g.cand[v] : (int)gc_k8_cand(b);
                gc_commit_colour(g, (int)v, cc);
                if (want_cround) g.cround[v] = round;
                lmaxc = cc > lmaxc ? cc : lmaxc;
                lacc++;
                tstart = g.trp[v];
                din = (int)(g.trp[v + 1] - tstart);
            }
            s_start[w][lane] = tstart;
            const int incl = gc_wave_incl_scan(din);
            const int excl = incl - din;
            const int total = __shfl(incl, GC_WAVE - 1, GC_WAVE);
            gc_wave_sync();
            for (int base = 0; base < total; base += GC_WAVE) {
                const int e = base + lane;
                const int o = gc_owner(excl, e);
                const int eo = __shfl(excl, o, GC_WAVE);
                bool claim = false;
                int x = 0;
                if (e < total) {
                    x = g.tcol[s_start[w][o] + (e - eo)];
                    claim = gc_claim(g.inF, x);
                }
                gc_stage_push(st, claim, x, next, next_cnt);
            }
            gc_wave_sync();
            if (g.hbits_w) gc_hub_push_wave(g, win, (int)v, cc, s_start[w], s_cc[w], big, &c->list_cnt);
        }
    }
    gc_stage_flush_block(st, next, next_cnt);
    __syncthreads();
    gc_block_max(&c->maxcolor, lmaxc, (long long*)scratch);
    gc_block_add(&c->accepted, lacc, scratch);
}

// A seam's send buffer, built on the device (no host round trip): HDR header words -- the
// rank's round scalars, encoded as (0xFFFFFFFF << 32 | value) so every delta applier reads
// them as padding -- then up to cap of the phase's deltas, padded with -1.
//   kind GC_KIND_CAND  (propose seam): frontier, max candidate, #candidates >= k, #deltas,
//                      winners of the last finished round (-halt code when it halted)
//   kind GC_KIND_STATE (sweep seam):   undecided (lists of slot `slot`), #deltas, undecided lights, #deltas, 0
// With delta == null only the header is written (the slice seams).
__device__ __forceinline__ long long gc_hdr_word(long long x) {
    return (long long)((0xFFFFFFFFull << 32) | (ull)(unsigned)x);
}
__global__ void __launch_bounds__(GC_BLOCK) k_shard_pack(GDev g, int kind, int slot, const long long* delta,
                                                         long long* send, long long cap) {
    const DevCtl* c = g.ctl;
    // (replicated hubs: the proposal deltas are compacted, k_delta_cand)
    const long long cnt = kind == GC_KIND_CAND && !g.hub_repl ? (long long)c->fcnt[c->cur] : (long long)c->dcnt;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        long long h[GC_SEAM_HDR];
        if (kind == GC_KIND_CAND) {
            h[0] = (long long)(c->fcnt[c->cur] - c->xhub_cnt);  // the rank's own frontier
            h[1] = c->maxmex;
            h[2] = (long long)c->failcnt;
            h[3] = cnt;
            h[4] = c->halt ? -(long long)c->halt : c->acc_last;
        } else {
            // (+ hubs waiting for every rank's lights: gc_shard_start_hubs decides them)
            h[0] = (long long)(c->und_cnt[slot] + c->undh_cnt[slot]) +
                   (g.hub_w && c->hub_start == GC_HUB_NOT_STARTED ? (long long)c->heavy_cnt : 0ll);
            h[1] = cnt;
            h[2] = (long long)c->und_cnt[slot];  // undecided lights (every rank's 0: the hubs start)
            h[3] = cnt;
            h[4] = 0;
        }
        for (int i = 0; i < GC_SEAM_HDR; ++i) send[i] = gc_hdr_word(h[i]);
    }
    if (!delta) return;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (long long)gridDim.x * blockDim.x)
        send[GC_SEAM_HDR + i] = i < cnt ? delta[i] : -1ll;
}

// per-round counter reset of a shard (one thread)
__global__ void k_shard_reset(GDev g, long long round) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    DevCtl* c = g.ctl;
    if (c->halt == GC_H_SWEEPS) return;  // the last finish halted: everything stays for gc_shard_resume_hubs
    if (c->loop_err == GC_LERR_LIST) return;  // a list overflowed: stay halted (shard_sync reports it)
    if (c->acc_round != round + 1) {  // a repeated seam (after a hub halt) keeps the first reset's count:
        c->acc_last = (long long)c->accepted;  // `accepted` was zeroed by it
        c->acc_round = round + 1;
    }
    c->halt = GC_RUN;
    c->round = round;
    c->heavy_cnt = 0;
    c->wide_cnt = 0;
    c->failcnt = 0;
    c->accepted = 0;
    c->maxmex = -1;
    c->sweeps = 0;
    c->dcnt = 0;
    c->rwin_cnt = 0;
    c->bigw_cnt = 0;
    c->list_cnt = 0;
    c->seed_cnt[0] = 0;
    c->seed_cnt[1] = 0;
    c->xhub_cnt = 0;
    c->lights_hold = g.hub_w ? 1 : 0;
    c->hub_start = GC_HUB_NOT_STARTED;
    for (int k = 0; k < 3; ++k) {
        c->und_cnt[k] = 0;
        c->undh_cnt[k] = 0;
    }
}

// Shards with replicated hubs: every uncoloured hub that a winner of any rank touched
// (hseen, set by gc_hub_mark) joins this rank's frontier list `slot` (a hub is in the
// frontier iff it has a coloured listed neighbour: coloring.py:86-95); the claim bitmap
// keeps every hub listed once.
__global__ void __launch_bounds__(GC_BLOCK) k_shard_hub_claim(GDev g, GLists L, int slot_next) {
    DevCtl* c = g.ctl;
    if (c->halt) return;
    __shared__ int s_stage[GC_WAVES_PER_BLOCK][GC_STAGE_CAP];
    const int w = threadIdx.x / GC_WAVE;
    const int slot = slot_next ? (c->cur ^ 1) : c->cur;
    GcStage st{s_stage[w], 0, g.list_cap, &g.ctl->loop_err, &g.ctl->halt};
    const long long H = g.nhub_repl;
    const long long steps = (H + GC_WAVE - 1) / GC_WAVE;
    for (long long sidx = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w; sidx < steps;
         sidx += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
        const long long x = sidx * GC_WAVE + gc_lane();
        bool claim = false;
        int v = 0;
        if (x < H && g.hseen[x]) {
            v = g.hub_v[x];
            claim = g.c8[v] == GC_C8_NONE && gc_claim(g.inF, v);
        }
        gc_stage_push(st, claim, v, L.F[slot], &c->fcnt[slot]);
    }
    gc_stage_flush_block(st, L.F[slot], &c->fcnt[slot]);
}

// Replicated hubs after a slice seam moved light states without deltas: every other rank's
// light winner flags the hubs listing it that propose its colour (what k_apply does for the
// state deltas, and a local winner in its sweep).  Flags are idempotent.
__global__ void __launch_bounds__(GC_BLOCK) k_shard_hub_flags(GDev g, long long lo, long long hi) {
    const long long n = g.n;
    for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (long long)gridDim.x * blockDim.x) {
        if (v >= lo && v < hi) continue;
        const unsigned kv = g.k8[v];
        if (gc_k8_state(kv) != GC_JP_IN || gc_k8_cand(kv) == GC_K8_NONE || g.hid[v] >= 0) continue;
        const int cv = gc_k8_cand(kv) == GC_K8_BIG ? g.cand[v] : (int)gc_k8_cand(kv);
        for (long long e = g.hin_rp[v]; e < g.hin_rp[v + 1]; ++e) {
            const int hx = g.hin_col[e];
            if ((g.hk[hx] >> 2) == (unsigned)cv && !g.hkill[hx]) g.hkill[hx] = 1u;
        }
    }
}

// after the push: the next frontier becomes current, the old slot becomes the output
__global__ void k_shard_flip(GDev g) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    DevCtl* c = g.ctl;
    if (c->halt) return;
    c->fcnt[c->cur] = 0;
    c->cur ^= 1;
}

// ------------------------------------------------------------------------------------
// E1 re-seed: components of the uncoloured-induced subgraph (lock-free union-find,
// parents always point to smaller positions), one argmax-(deg,pos) seed per component.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ int cc_load(int* p, int x) {
    return __hip_atomic_load(&p[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int cc_find(int* p, int x) {
    int q = cc_load(p, x);
    while (q != x) {
        x = q;
        q = cc_load(p, x);
    }
    return x;
}

__global__ void __launch_bounds__(GC_BLOCK) k_unc_compact(GDev g, int* list, ull* list_cnt, int* parent,
                                                          ull* best) {
    __shared__ int s_stage[GC_WAVES_PER_BLOCK][GC_STAGE_CAP];
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    GcStage st{s_stage[w], 0, g.list_cap, &g.ctl->loop_err, &g.ctl->halt};
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v - lane < g.n; v += stride) {
        const bool u = v < g.n && g.c8[v] == GC_C8_NONE;
        if (u) {
            parent[v] = (int)v;
            best[v] = 0;
        }
        gc_stage_push(st, u, (int)v, list, list_cnt);
    }
    gc_stage_flush(st, list, list_cnt);
}

__global__ void __launch_bounds__(GC_BLOCK) k_cc_hook(GDev g, const int* list, const ull* list_cnt, int* parent) {
    __shared__ long long s_start[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_v[GC_WAVES_PER_BLOCK][GC_WAVE];
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    const long long cnt = (long long)*list_cnt;
    for (long long chunk = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w; chunk * GC_WAVE < cnt;
         chunk += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
        const long long idx = chunk * GC_WAVE + lane;
        const int v = idx < cnt ? list[idx] : -1;
        const int d = v >= 0 ? g.deg[v] : 0;
        s_start[w][lane] = v >= 0 ? g.rp[v] : 0;
        s_v[w][lane] = v;
        const int incl = gc_wave_incl_scan(d);
        const int excl = incl - d;
        const int total = __shfl(incl, GC_WAVE - 1, GC_WAVE);
        gc_wave_sync();
        for (int base = 0; base < total; base += GC_WAVE) {
            const int e = base + lane;
            const int o = gc_owner(excl, e);
            const int eo = __shfl(excl, o, GC_WAVE);
            if (e < total) {
                const int u = g.col[s_start[w][o] + (e - eo)];
                int a = s_v[w][o];
                if (u != a && g.c8[u] == GC_C8_NONE) {
                    int b = u;
                    while (true) {
                        a = cc_find(parent, a);
                        b = cc_find(parent, b);
                        if (a == b) break;
                        if (a > b) { const int t = a; a = b; b = t; }
                        if (atomicCAS(&parent[b], b, a) == b) break;
                    }
                }
            }
        }
        gc_wave_sync();
    }
}

__global__ void __launch_bounds__(GC_BLOCK) k_cc_best(GDev g, const int* list, const ull* list_cnt, int* parent,
                                                      ull* best) {
    const long long cnt = (long long)*list_cnt;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += (long long)gridDim.x * blockDim.x) {
        const int v = list[i];
        const int r = cc_find(parent, v);
        atomicMax(&best[r], ((ull)g.deg[v] << 32) | (ull)v);
    }
}

__global__ void __launch_bounds__(GC_BLOCK) k_cc_seeds(GDev g, const int* list, const ull* list_cnt, int* parent,
                                                       const ull* best, int* seed_light, int* seed_heavy) {
    const long long cnt = (long long)*list_cnt;
    const int lane = gc_lane();
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i - lane < cnt; i += stride) {
        const int v = i < cnt ? list[i] : -1;
        const bool root = v >= 0 && cc_load(parent, v) == v;
        int s = -1, d = 0;
        if (root) {
            s = (int)(best[v] & 0xFFFFFFFFull);
            d = g.deg[s];
            g.k8[s] = gc_k8(0u, GC_JP_IN);
            atomicOr(&g.inF[s >> 5], 1u << (s & 31));
        }
        gc_wave_append(root && d > GC_HEAVY_T, s, seed_heavy, &g.ctl->seed_cnt[1]);
        gc_wave_append(root && d <= GC_HEAVY_T, s, seed_light, &g.ctl->seed_cnt[0]);
    }
}

// ------------------------------------------------------------------------------------
// validate_graph_coloring counts (coloring.py:149-162)
// ------------------------------------------------------------------------------------
// Final colours from the byte mirror (colours >= 254 were stored directly).
__global__ void __launch_bounds__(GC_BLOCK) k_finalize(GDev g) {
    for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < g.n;
         v += (long long)gridDim.x * blockDim.x) {
        const unsigned b = g.c8[v];
        if (b != GC_C8_BIG) g.color[v] = b == GC_C8_NONE ? -1 : (int)b;
    }
}

// ------------------------------------------------------------------------------------
// Resume (gc_color_resume): the engine's state at the start of round `round0` from a
// colouring in progress -- the multi-GPU hybrid hands the replicated colours and the
// all-gathered frontier of its sharded rounds to the one-GPU engine for the rest.  The
// state is exactly what the engine keeps at a round start: colours (c8 / color / cround),
// k8 cleared, the claim bitmap = coloured or in the frontier, the frontier list, the hub
// mirror and forbidden-colour bitmaps (every coloured vertex pushes its colour into the hubs
// that list it, as its commit did), U and the max colour.
// ------------------------------------------------------------------------------------
__global__ void __launch_bounds__(GC_BLOCK) k_resume_init(GDev g, const int* colors, const int* cround_in) {
    __shared__ ull scratch[2 * GC_WAVES_PER_BLOCK];
    const int lane = gc_lane();
    ull unc = 0;
    long long mx = -1;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v - lane < g.n; v += stride) {
        const bool valid = v < g.n;
        const int c = valid ? colors[v] : 0;
        const bool coloured = valid && c >= 0;
        if (valid) {
            g.color[v] = coloured ? c : -1;
            g.cround[v] = cround_in ? cround_in[v] : (coloured ? 0 : -1);
            g.c8[v] = gc_c8_of(coloured ? (long long)c : -1ll);
            g.k8[v] = gc_k8(GC_K8_NONE, GC_JP_UND);
            if (g.hub_w && g.hid[v] >= 0) g.hk[g.hid[v]] = coloured ? GC_HK_COLOURED : gc_hk(GC_HK_NOCAND, GC_JP_UND);
            g.mark[v] = 0;
            if (coloured) mx = c > mx ? c : mx;
            else unc++;
        }
        const ull m = __ballot(coloured || !valid);  // claim bitmap: coloured (frontier bits: k_resume_front)
        if (lane == 0) {
            const long long w = (v - lane) >> 5;
            g.inF[w] = (unsigned)m;
            if ((v - lane) + 32 < g.n) g.inF[w + 1] = (unsigned)(m >> 32);
        }
    }
    gc_block_max(&g.ctl->maxcolor, mx, (long long*)scratch);
    gc_block_add(&g.ctl->uncolored, unc, scratch);
}

// the frontier list F[0] and its claim bits (after k_resume_init's bitmap words).  An entry
// out of [0, n) is the caller's error: it is listed as vertex 0 (never read through) and
// loop_err 4 makes k_resume_close stop the run before any round, and the host report it.
__global__ void __launch_bounds__(GC_BLOCK) k_resume_front(GDev g, GLists L, const int* front, long long nf) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nf; i += (long long)gridDim.x * blockDim.x) {
        int v = front[i];
        if (v < 0 || v >= g.n) {
            __hip_atomic_store(&g.ctl->loop_err, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v = 0;
        }
        L.F[0][i] = v;
        atomicOr(&g.inF[v >> 5], 1u << (v & 31));
    }
}

// every coloured vertex's colour into the bitmaps of the hubs that list it (lists longer
// than GC_PUSH_FLAT go to `big` for gcl_hub_push_big, as in the commits)
__global__ void __launch_bounds__(GC_BLOCK) k_resume_hbits(GDev g, const int* colors, int* big, ull* big_cnt) {
    __shared__ long long s_start[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_cc[GC_WAVES_PER_BLOCK][GC_WAVE];
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    const long long steps = (g.n + GC_WAVE - 1) / GC_WAVE;
    for (long long sidx = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w; sidx < steps;
         sidx += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
        const long long v = sidx * GC_WAVE + lane;
        const int c = v < g.n ? colors[v] : -1;
        gc_hub_push_wave(g, c >= 0, (int)v, c, s_start[w], s_cc[w], big, big_cnt);
    }
}

// U and the start-of-round checks (one thread): U == 0 ends the colouring, an empty frontier
// with uncoloured vertices left asks for E1 (or stalls with E1 off), as after any round
__global__ void k_resume_close(GDev g, GLists L) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    DevCtl* c = g.ctl;
    if (c->loop_err == 4) {  // a frontier entry out of range (k_resume_front): no round runs
        gc_st(&c->halt, (int)GC_H_DONE);
        return;
    }
    const long long U = (long long)c->uncolored;
    gc_st(&c->U, U);
    gc_precheck(L, c, U, (long long)c->fcnt[c->cur]);
}

// a shard's own frontier (F[cur] minus the replicated hubs it lists but does not own)
__global__ void __launch_bounds__(GC_BLOCK) k_shard_own_front(GDev g, GLists L, long long lo, long long hi, int* out,
                                                              ull* out_cnt) {
    DevCtl* c = g.ctl;
    const int cur = c->cur;
    const long long cnt = (long long)c->fcnt[cur];  // (includes the replicated hubs of other ranks)
    const int* list = L.F[cur];
    const long long steps = (cnt + GC_WAVE - 1) / GC_WAVE;
    const int w = threadIdx.x / GC_WAVE;
    for (long long sidx = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w; sidx < steps;
         sidx += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
        const long long i = sidx * GC_WAVE + gc_lane();
        const int v = i < cnt ? list[i] : -1;
        gc_wave_append(v >= lo && v < hi && g.c8[v] == GC_C8_NONE, v, out, out_cnt);
    }
}

// ------------------------------------------------------------------------------------
// graph helpers
// ------------------------------------------------------------------------------------
// deg, its byte key kb = gc_deg_code(deg) (the rank partition gathers it first: gc_prep.hip),
// the max degree; *bad counts violations of the CSR offset contract
__global__ void k_degrees(const long long* rp, int n, long long nnz, int* deg, unsigned char* kb, ull* maxdeg, ull* bad) {
    ull m = 0, b = 0;
    for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (long long)gridDim.x * blockDim.x) {
        const long long d = rp[v + 1] - rp[v];
        deg[v] = (int)d;
        kb[v] = (unsigned char)gc_deg_code(d);
        m = (d > 0 && (ull)d > m) ? (ull)d : m;
        b += d < 0;
        if (v == 0) b += rp[0] != 0;
        if (v == n - 1) b += rp[n] != nnz;
    }
    m = gc_wave_max(m);
    b = gc_wave_sum(b);
    if (gc_lane() == 0) {
        if (m) atomicMax(maxdeg, m);
        if (b) atomicAdd(bad, b);
    }
}

// ------------------------------------------------------------------------------------
// host-callable launch wrappers
// ------------------------------------------------------------------------------------
void gcl_init(const GDev& g, int* seed_light, int grid, hipStream_t s) {
    GC_LAUNCH(k_init, dim3(grid), dim3(GC_BLOCK), 0, s, g, seed_light);
}
void gcl_seed_prep(const GDev& g, int* sl, int* sh, hipStream_t s) {
    GC_LAUNCH(k_seed_prep, dim3(1), dim3(64), 0, s, g, sl, sh);
}
int gcl_fsort_blocks(long long n) { return (int)(((n + 31) / 32 + GC_BLOCK - 1) / GC_BLOCK); }
void gcl_fsort(const GDev& g, const GLists& L, unsigned* bsum, hipStream_t s) {
    const int nb = gcl_fsort_blocks(g.n);
    if (nb <= 0) return;
    GC_LAUNCH(k_fsort_count, dim3(nb), dim3(GC_BLOCK), 0, s, g, bsum);
    GC_LAUNCH(k_fsort_scan, dim3(1), dim3(1024), 0, s, g, bsum, nb, 0);
    GC_LAUNCH(k_fsort_write, dim3(nb), dim3(GC_BLOCK), 0, s, g, (const unsigned*)bsum, L, 0);
}
void gcl_front_build(const GDev& g, const GLists& L, unsigned* bsum, hipStream_t s) {
    const int nb = gcl_fsort_blocks(g.n);
    if (nb <= 0) return;
    GC_LAUNCH(k_front_count, dim3(nb), dim3(GC_BLOCK), 0, s, g, bsum);
    GC_LAUNCH(k_fsort_scan, dim3(1), dim3(1024), 0, s, g, bsum, nb, 1);
    GC_LAUNCH(k_fsort_write, dim3(nb), dim3(GC_BLOCK), 0, s, g, (const unsigned*)bsum, L, 1);
}
// Grids of the gather-heavy round kernels (workgroups; they grid-stride over device
// counts).  Their waves spend ~80% of their cycles waiting on gathers (SQ_WAIT_ANY), so
// the grid sets how many are in flight; GC_GRID_{P,R,C} override for measurements.
static int round_grid(const char* env, int dflt) {
    const char* e = getenv(env);
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : dflt;
}
static const int kGridP = round_grid("GC_GRID_P", GC_ROUND_GRID);
// k_propose when the last snapshot's frontier was small (< n/256): 512 workgroups (R-MAT-24
// 216 -> 210 ms with the later sweeps on 256; the full grid stays for C2's big rounds)
static const int kGridPS = round_grid("GC_GRID_PS", 512);
static const int kGridR = round_grid("GC_GRID_R", GC_ROUND_GRID);
// (round 3's GC_GRID_SMALL -- resolve / commit / commit_big capped to 256 workgroups in small
// rounds -- measured R-MAT-24 -0.1%, C2 +2% in round 4, profiles/r04/c: removed)
static const int kGridC = round_grid("GC_GRID_C", 768);  // mesh 512^3 111 -> 106 ms (1024 -> 768; 1536: 158), R-MAT and C2 alike
static const int kGridPB = round_grid("GC_GRID_PB", GC_BLOCK_GRID);  // k_propose_block
static const int kGridCB = round_grid("GC_GRID_CB", GC_ROUND_GRID);  // k_commit_big
// the later JP sweeps: mostly short lists, where 1024 workgroups' start-up and end-of-kernel
// reductions outweigh their reach (R-MAT-24 257 -> 238 ms, R-MAT-26 562 -> 521 ms at 384;
// 256 within 1%; C2 and the mesh unchanged)
static const int kGridS = round_grid("GC_GRID_S", 256);
// ... when heavy vertices are resolved a workgroup each (no hub JP: seeded ranks, hubs off):
// seeded R-MAT-24 1520 ms on 256 workgroups, 1265 on 384, 938 on 1024
static const int kGridSH = round_grid("GC_GRID_SH", 1024);
// ... and the first sweep (k_resolve) then: seeded R-MAT-24 935 ms on 1024, 879 on 2048, 862 on 4096
static const int kGridRH = round_grid("GC_GRID_RH", 4096);

// per-slot stats -> DevCtl.sumdeg / nvert (one workgroup; before the host reads them)
__global__ void k_stat_reduce(GDev g) {
    const int t = threadIdx.x;
    if (t < 16) {
        ull a = 0;
        for (int k = 0; k < GC_STAT_SLOTS; ++k) a += g.bstat[k * 16 + t];
        if (t < 8) g.ctl->sumdeg[t] = a;
        else g.ctl->nvert[t - 8] = a;
    }
}
void gcl_stat_reduce(const GDev& g, hipStream_t s) {
    GC_LAUNCH(k_stat_reduce, dim3(1), dim3(64), 0, s, g);
}

void gcl_pack_c4(const GDev& g, hipStream_t s) {
    GC_LAUNCH(k_pack_c4, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, g);
}
void gcl_propose(const GDev& g, const GLists& L, hipStream_t s, int small, int inl) {
    if (inl) GC_LAUNCH(k_propose<1>, dim3(small ? kGridPS : kGridP), dim3(GC_BLOCK), 0, s, g, L);
    else GC_LAUNCH(k_propose<0>, dim3(small ? kGridPS : kGridP), dim3(GC_BLOCK), 0, s, g, L);
}
void gcl_propose_block(const GDev& g, const GLists& L, hipStream_t s) {
    GC_LAUNCH(k_propose_block, dim3(kGridPB), dim3(GC_BLOCK), (size_t)GC_MEX_WORDS * 4, s, g, L);
}
void gcl_resolve(const GDev& g, const GLists& L, hipStream_t s) {
    GC_LAUNCH(k_resolve, dim3(g.heavy_wg ? kGridRH : kGridR), dim3(GC_BLOCK), 0, s, g, L);
}
void gcl_sweep(const GDev& g, const GLists& L, int i, hipStream_t s) {
    GC_LAUNCH(k_sweep, dim3(g.heavy_wg ? kGridSH : kGridS), dim3(GC_BLOCK), 0, s, g, L, i);
}
void gcl_delta_cand(const GDev& g, const GLists& L, hipStream_t s) {
    GC_LAUNCH(k_delta_cand, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, g, L);
}
void gcl_apply(const GDev& g, int kind, const long long* recv, long long count, long long lo, long long hi, int round,
               int* rwin, hipStream_t s, long long hdr_stride) {
    if (count <= 0) return;
    GC_LAUNCH(k_apply, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, g, kind, recv, count, lo, hi, round, rwin,
                       hdr_stride);
}
__global__ void k_shard_clear_halt(GDev g, int code) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && g.ctl->halt == code) g.ctl->halt = GC_RUN;
}
void gcl_shard_clear_halt(const GDev& g, int code, hipStream_t s) {
    GC_LAUNCH(k_shard_clear_halt, dim3(1), dim3(64), 0, s, g, code);
}
void gcl_shard_list_commit(const GDev& g, const GLists& L, const int* rwin, int* big, hipStream_t s) {
    GC_LAUNCH(k_shard_list_commit, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, g, L, rwin, big);
}
void gcl_shard_scan_commit(const GDev& g, const GLists& L, long long lo, long long hi, int* big, hipStream_t s) {
    GC_LAUNCH(k_shard_scan_commit, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, g, L, lo, hi, big);
}
void gcl_shard_pack(const GDev& g, int kind, int slot, const long long* delta, long long* send, long long cap,
                    hipStream_t s) {
    const int grid = (int)std::max<long long>(1, std::min<long long>((cap + GC_BLOCK - 1) / GC_BLOCK, 64));
    GC_LAUNCH(k_shard_pack, dim3(grid), dim3(GC_BLOCK), 0, s, g, kind, slot, delta, send, cap);
}
void gcl_shard_reset(const GDev& g, long long round, hipStream_t s) {
    GC_LAUNCH(k_shard_reset, dim3(1), dim3(64), 0, s, g, round);
}
void gcl_shard_hub_claim(const GDev& g, const GLists& L, int slot_next, hipStream_t s) {
    if (g.hub_repl && g.nhub_repl > 0)
        GC_LAUNCH(k_shard_hub_claim, dim3((int)std::min<long long>((g.nhub_repl + GC_BLOCK - 1) / GC_BLOCK, 2048)), dim3(GC_BLOCK), 0, s, g, L, slot_next);
}
void gcl_shard_hub_flags(const GDev& g, long long lo, long long hi, hipStream_t s) {
    if (g.hub_repl && g.hub_w && g.n > 0)
        GC_LAUNCH(k_shard_hub_flags, dim3((int)std::min<long long>((g.n + GC_BLOCK - 1) / GC_BLOCK, 2048)), dim3(GC_BLOCK), 0, s, g, lo, hi);
}
void gcl_shard_flip(const GDev& g, hipStream_t s) { GC_LAUNCH(k_shard_flip, dim3(1), dim3(64), 0, s, g); }
// the winners gc_hub_push_wave left in `big`: their hub lists as one flat range over the
// whole grid, GC_BLOCK winners at a time (every workgroup scans the tile's list lengths and
// takes its stride of the tile's entries), 4 entries per thread in flight.  (Round 3 gave
// each winner a workgroup: a hub's list of 10^4-10^5 hubs was then one workgroup's chain of
// dependent load-load-atomic steps, ~100 us a round in variant B, profiles/r04/f.)
#ifndef GC_PUSH_BIG_WG
#define GC_PUSH_BIG_WG 0  // build knob for the A/B: 1 = round 3's workgroup per winner
#endif
#if GC_PUSH_BIG_WG
__global__ void __launch_bounds__(GC_BLOCK) k_hub_push_big(GDev g, const int* big, const ull* cnt) {
    const long long nb = (long long)*cnt;
    for (long long i = blockIdx.x; i < nb; i += gridDim.x) {
        const int v = big[i];
        gc_hub_mark_row(g, v, gc_colour(g, v), threadIdx.x, blockDim.x);
    }
}
#else
__global__ void __launch_bounds__(GC_BLOCK) k_hub_push_big(GDev g, const int* big, const ull* cnt) {
    const long long nb = (long long)*cnt;
    if (nb == 0) return;
    __shared__ long long s_off[GC_BLOCK + 1];
    __shared__ long long s_hs[GC_BLOCK];
    __shared__ int s_cc[GC_BLOCK];
    __shared__ long long s_wsum[GC_WAVES_PER_BLOCK];
    const int t = threadIdx.x, lane = gc_lane(), w = t / GC_WAVE;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long j0 = 0; j0 < nb; j0 += GC_BLOCK) {
        const int tn = (int)(nb - j0 < GC_BLOCK ? nb - j0 : GC_BLOCK);
        long long len = 0;
        if (t < tn) {
            const int v = big[j0 + t];
            s_hs[t] = g.hin_rp[v];
            len = g.hin_rp[v + 1] - s_hs[t];
            s_cc[t] = gc_colour(g, v);  // committed: its colour is in c8
        }
        long long x = len;  // workgroup inclusive scan of len
#pragma unroll
        for (int o = 1; o < GC_WAVE; o <<= 1) {
            const long long y = __shfl_up(x, o, GC_WAVE);
            if (lane >= o) x += y;
        }
        if (lane == GC_WAVE - 1) s_wsum[w] = x;
        __syncthreads();
        for (int k = 0; k < w; ++k) x += s_wsum[k];
        s_off[t + 1] = x;
        if (t == 0) s_off[0] = 0;
        __syncthreads();
        const long long total = s_off[tn];
        for (long long f0 = (long long)blockIdx.x * blockDim.x * 4; f0 < total; f0 += stride * 4) {
            int hx[4], hc[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const long long f = f0 + (long long)q * blockDim.x + t;
                hx[q] = -1;
                hc[q] = 0;
                if (f < total) {
                    int k = 0;  // max k < tn with s_off[k] <= f
#pragma unroll
                    for (int step = GC_BLOCK / 2; step > 0; step >>= 1)
                        if (k + step < tn && s_off[k + step] <= f) k += step;
                    hx[q] = g.hin_col[s_hs[k] + (f - s_off[k])];
                    hc[q] = s_cc[k];
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (hx[q] >= 0) gc_hub_mark(g, hx[q], hc[q]);
        }
        __syncthreads();
    }
}
#endif
#ifdef GC_A_PROF
// append this colouring's per-round k_sweep_async records (GC_A_PROF_OUT) and clear them
void gcl_aprof_dump(const RoundRec* recs, size_t nrec) {
    const char* pp = getenv("GC_A_PROF_OUT");
    if (!pp) return;
    static ull hb[GC_A_PROF_ROUNDS][GC_A_PROF_K];
    if (hipMemcpyFromSymbol(hb, HIP_SYMBOL(gc_aprof), sizeof(hb)) != hipSuccess) return;
    if (FILE* f = fopen(pp, "a")) {
        fprintf(f, "# colouring: %zu rounds; per round: r U F light_end_us light_wait_end_us hub_end_us max_lpass max_hpass "
                   "lights hubs sum_lpass light_waves max_wave_lights sum_hpass max_wave_hubs hub_scanned max_hub_scan hubs_in "
                   "hub_remaining\n", nrec);
        for (size_t i = 0; i < nrec && i < GC_A_PROF_ROUNDS; ++i) {
            const ull* r = hb[i];
            fprintf(f, "%zu %lld %lld %.2f %.2f %.2f %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu\n", i,
                    recs[i].U, recs[i].F, r[0] / 100.0, r[1] / 100.0, r[2] / 100.0, r[3], r[4], r[5], r[6], r[7], r[8], r[9],
                    r[10], r[11], r[12], r[13], r[14], r[15]);
        }
        gcl_cprof_dump(f, nrec);
        fclose(f);
    }
    static ull z[GC_A_PROF_ROUNDS][GC_A_PROF_K];
    (void)hipMemcpyToSymbol(HIP_SYMBOL(gc_aprof), z, sizeof(z));
}
#endif
void gcl_hub_push_big(const GDev& g, const int* big, const ull* cnt, hipStream_t s) {
    GC_LAUNCH(k_hub_push_big, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, g, big, cnt);
}
void gcl_close(const GDev& g, const GLists& L, int mode, hipStream_t s, int allow_big, int fused, DevCtl* snap) {
    GC_LAUNCH(k_close, dim3(1), dim3(64), 0, s, g, L, mode, allow_big, fused, snap);
}
void gcl_resume(const GDev& g, const GLists& L, const int* colors, const int* cround, const int* front, long long nf,
                int* big, ull* big_cnt, hipStream_t s) {
    const int grid = (int)std::max<long long>(1, std::min<long long>((g.n + GC_BLOCK - 1) / GC_BLOCK, 8192));
    GC_LAUNCH(k_resume_init, dim3(grid), dim3(GC_BLOCK), 0, s, g, colors, cround);
    if (nf > 0)
        GC_LAUNCH(k_resume_front, dim3((int)std::max<long long>(1, std::min<long long>((nf + GC_BLOCK - 1) / GC_BLOCK, 8192))),
                           dim3(GC_BLOCK), 0, s, g, L, front, nf);
    if (g.hbits_w) {
        GC_LAUNCH(k_resume_hbits, dim3(grid), dim3(GC_BLOCK), 0, s, g, colors, big, big_cnt);
        gcl_hub_push_big(g, big, big_cnt, s);
    }
    GC_LAUNCH(k_resume_close, dim3(1), dim3(64), 0, s, g, L);
}
void gcl_shard_own_front(const GDev& g, const GLists& L, long long lo, long long hi, int* out, ull* out_cnt,
                         hipStream_t s) {
    GC_LAUNCH(k_shard_own_front, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, g, L, lo, hi, out, out_cnt);
}
// the control block into a host-mapped snapshot slot (variant B's per-round wait: a kernel's
// vector stores instead of a copy-engine blit)
__global__ void k_snap_ctl(DevCtl* c, DevCtl* snap) { gc_snap_copy(c, snap); }
void gcl_snap(DevCtl* ctl, DevCtl* snap, hipStream_t s) { GC_LAUNCH(k_snap_ctl, dim3(1), dim3(GC_BLOCK), 0, s, ctl, snap); }
void gcl_finalize(const GDev& g, int grid, hipStream_t s) {
    GC_LAUNCH(k_finalize, dim3(grid), dim3(GC_BLOCK), 0, s, g);
}
void gcl_sweep_loop(const GDev& g, const GLists& L, int S, int grid, hipStream_t s) {
    GC_LAUNCH(k_sweep_loop, dim3(grid), dim3(GC_BLOCK), 0, s, g, L, S);
}
void gcl_sweep_tail(const GDev& g, const GLists& L, int S, hipStream_t s) {
    if (g.tail_nw == 16) GC_LAUNCH(k_sweep_tail<16>, dim3(1), dim3(16 * GC_WAVE), 0, s, g, L, S);
    else if (g.tail_nw == 8) GC_LAUNCH(k_sweep_tail<8>, dim3(1), dim3(8 * GC_WAVE), 0, s, g, L, S);
    else GC_LAUNCH(k_sweep_tail<4>, dim3(1), dim3(4 * GC_WAVE), 0, s, g, L, S);
}
void gcl_sweep_async(const GDev& g, const GLists& L, int S, int par, long long budget, int grid, hipStream_t s,
                     int lds_lights) {
    // the lights' LDS rows (GC_LIGHT_LDS) as dynamic LDS, only where the host asks for them
    // (big rounds): 28 KB more per workgroup slowed the small rounds' launches (profiles/r06/r)
    const size_t dyn = (GC_LIGHT_LDS && lds_lights) ? sizeof(GcLightLds) * GC_WAVES_PER_BLOCK : 0;
    GC_LAUNCH(k_sweep_async, dim3(grid), dim3(GC_BLOCK), dyn, s, g, L, S, par, budget, dyn ? 1 : 0);
}
int gc_resident_blocks_per_cu(const void* fn, int block) {
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, block, 0) != hipSuccess) return 0;
    hipFuncAttributes a;
    if (hipFuncGetAttributes(&a, fn) == hipSuccess && a.numRegs > 0) {
        const int vg = (a.numRegs + 7) / 8 * 8;
        const int waves_simd = std::min(8, 512 / vg);
        const int waves_block = (block + GC_WAVE - 1) / GC_WAVE;
        int by_regs = waves_simd * 4 / waves_block;  // 4 SIMDs per CU
        if (a.sharedSizeBytes > 0) by_regs = std::min(by_regs, (int)((160u << 10) / a.sharedSizeBytes));
        occ = std::min(occ, by_regs);
    }
    return occ;
}
int gcl_sweep_async_blocks_per_cu() { return gc_resident_blocks_per_cu((const void*)k_sweep_async, GC_BLOCK); }

// Resident workgroups per CU of a kernel with a residency-probe mode, measured once per
// device and cached (gc_residency_probe; `launch` starts the kernel in probe mode on `grid`
// workgroups).  The control block's async_done words are used and zeroed again.
int gc_measure_resident(const void* key, gc_graph_ctl_view v, int query, void (*launch)(const GDev&, int, hipStream_t)) {
    static std::mutex mu;
    static std::map<std::pair<const void*, int>, int> cache;
    int dev = 0;
    hipGetDevice(&dev);
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache.find({key, dev});
        if (it != cache.end()) return it->second;
    }
    int cus = 0;
    if (query <= 0 || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return query;
    const int grid = cus * std::min(8, query + 1);  // one more per CU than the runtime allows
    // A process's first launches of a kernel can dispatch slowly enough that the probe's
    // 100-us window closes before every resident workgroup arrived (round 6 saw 256 of 2048 in
    // one process, and the grid would have stayed at 1 per CU for good): the probe
    // runs again while it reads below the runtime's answer, and the largest reading counts.
    ull best = 0;
    for (int attempt = 0; attempt < 4 && best < (ull)cus * (ull)query; ++attempt) {
        ull r[2] = {0, 0};
        if (hipMemsetAsync(v.g->ctl->async_done, 0, sizeof(r), v.s) != hipSuccess) return std::max(1, query - 1);
        launch(*v.g, grid, v.s);
        if (hipMemcpyAsync(r, v.g->ctl->async_done, sizeof(r), hipMemcpyDeviceToHost, v.s) != hipSuccess ||
            hipMemsetAsync(v.g->ctl->async_done, 0, sizeof(r), v.s) != hipSuccess || hipStreamSynchronize(v.s) != hipSuccess)
            return std::max(1, query - 1);
        if (getenv("GC_DEBUG"))
            fprintf(stderr, "[gc] residency probe %d: %llu of %d workgroups resident at once (runtime answer %d per CU)\n",
                    attempt, r[1], grid, query);
        best = std::max(best, r[1]);
    }
    const int per_cu = std::max(1, std::min(query, (int)(best / (ull)cus)));
    if (getenv("GC_DEBUG")) fprintf(stderr, "[gc] residency: %d per CU\n", per_cu);
    std::lock_guard<std::mutex> lk(mu);
    cache[{key, dev}] = per_cu;
    return per_cu;
}
static void launch_sweep_async_probe(const GDev& g, int grid, hipStream_t s) {
    GLists L{};
    GC_LAUNCH(k_sweep_async, dim3(grid), dim3(GC_BLOCK), 0, s, g, L, 0, 0, -1ll, 0);
}
int gcl_sweep_async_resident(const GDev& g, hipStream_t s) {
    return gc_measure_resident((const void*)k_sweep_async, gc_graph_ctl_view{&g, s}, gcl_sweep_async_blocks_per_cu(),
                               launch_sweep_async_probe);
}
void gcl_pull(const GDev& g, int allow_big, hipStream_t s) {
    GC_LAUNCH(k_pull, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, g, allow_big);
}
void gcl_commit(const GDev& g, const GLists& L, int mode, int nsweeps, hipStream_t s, int allow_big, int fused,
                DevCtl* snap, int tclose) {
    const int gc = kGridC;
    if (fused) {  // no heavy vertex, so nothing is deferred to k_commit_big
        GC_LAUNCH(k_commit<1>, dim3(gc), dim3(GC_BLOCK), 0, s, g, L, mode, nsweeps, allow_big, snap, tclose);
        return;
    }
    // tclose 2: k_commit_big's last workgroup closes the round (k_commit does not)
    GC_LAUNCH(k_commit<0>, dim3(gc), dim3(GC_BLOCK), 0, s, g, L, mode, nsweeps, allow_big, tclose == 2 ? nullptr : snap,
              tclose == 2 ? 0 : tclose);
    if (g.big_rows)  // otherwise no in-row can exceed GC_BIGROW
        GC_LAUNCH(k_commit_big, dim3(kGridCB), dim3(GC_BLOCK), 0, s, g, L, mode, allow_big, tclose == 2 ? snap : nullptr,
                  tclose == 2 ? 1 : 0);
}
void gcl_unc_compact(const GDev& g, int* list, ull* cnt, int* parent, ull* best, int grid, hipStream_t s) {
    GC_LAUNCH(k_unc_compact, dim3(grid), dim3(GC_BLOCK), 0, s, g, list, cnt, parent, best);
}
void gcl_cc_hook(const GDev& g, const int* list, const ull* cnt, int* parent, int grid, hipStream_t s) {
    GC_LAUNCH(k_cc_hook, dim3(grid), dim3(GC_BLOCK), 0, s, g, list, cnt, parent);
}
void gcl_cc_best(const GDev& g, const int* list, const ull* cnt, int* parent, ull* best, int grid, hipStream_t s) {
    GC_LAUNCH(k_cc_best, dim3(grid), dim3(GC_BLOCK), 0, s, g, list, cnt, parent, best);
}
void gcl_cc_seeds(const GDev& g, const int* list, const ull* cnt, int* parent, const ull* best, int* sl, int* sh,
                  int grid, hipStream_t s) {
    GC_LAUNCH(k_cc_seeds, dim3(grid), dim3(GC_BLOCK), 0, s, g, list, cnt, parent, best, sl, sh);
}
void gcl_degrees(const long long* rp, int n, long long nnz, int* deg, unsigned char* kb, ull* maxdeg, ull* bad, int grid,
                 hipStream_t s) {
    GC_LAUNCH(k_degrees, dim3(grid), dim3(GC_BLOCK), 0, s, rp, n, nnz, deg, kb, maxdeg, bad);
}
