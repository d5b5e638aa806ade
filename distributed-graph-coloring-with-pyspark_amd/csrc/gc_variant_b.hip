// gc_variant_b.hip -- variant B (coloring_optimized.py) on the GPU.
//
// Variant B differs from A in two places:
//   propose  every uncoloured vertex proposes; one with no coloured neighbour proposes 0
//            (coloring_optimized.py:150-166).  The frontier is therefore the whole
//            uncoloured set, rebuilt each round in vertex order by the frontier re-sort
//            kernels (DevCtl.fsort_all) instead of being pushed.
//   resolve  per candidate colour, an arrival-order (file-order) fold
//            (coloring_optimized.py:120-126, 168-200): an arriving v is admitted iff no
//            admitted u in N(v), u != v, has deg(u) >= deg(v); on admission v evicts every
//            admitted x of its group with v in N(x) and deg(x) < deg(v).
//
// The fold is sequential, but every decision only looks BACK in arrival order, so it is
// evaluated as a fixpoint of two monotone passes (dependency-ordered, like the JP sweeps
// of variant A):
//   adm(v)  UND -> IN (admitted at arrival) / OUT (refused).  v is refused as soon as one
//           earlier same-candidate neighbour u with deg(u) >= deg(v) is admitted and still
//           present when v arrives (ev(u) > v); admitted once every such u is known to be
//           refused or evicted before v.
//   ev(u)   for admitted u: the smallest position of a not-refused potential evictor
//           (v' in N(u), v' > u, same candidate, deg(v') > deg(u)); INF if none.  Refusals
//           only raise it, so a stale value is a lower bound; it is final once that evictor
//           is admitted (u evicted at its arrival) or INF (u never evicted).
// The earliest undecided vertex always decides in the next pass, so the passes converge;
// the round's winners are the admitted vertices with ev = INF.  Checked bit for bit
// against oracle/gcolor_oracle.c (variant 1) and the golden vectors made by running the
// reference's coloring_optimized.py (tests/test_gpu_parity.py).
#include <string.h>

#include <algorithm>
#include <vector>

#include "gc_device.h"
#include "gc_engine.h"

#define GC_B_INF 0x7FFFFFFF

namespace {

__device__ __forceinline__ int b_cand(const GDev& g, int v, unsigned kv) {
    const unsigned c6 = gc_k8_cand(kv);
    return c6 == GC_K8_BIG ? g.cand[v] : (int)c6;
}

// same candidate as the owner (c6 / full value cv)
__device__ __forceinline__ bool b_same(const GDev& g, int u, unsigned ku, unsigned c6, int cv) {
    if (gc_k8_cand(ku) != c6) return false;
    return c6 != GC_K8_BIG || g.cand[u] == cv;
}

// per-round counter reset (one thread)
__global__ void k_b_reset(GDev g, long long round) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    DevCtl* c = g.ctl;
    // halted -- a list append overflowed (gc_stage_fits), or the previous round's
    // commit found the colouring done, failed or its fold unfinished (pipelined rounds,
    // k_b_commit): this round is a no-op, every kernel of it returns at once, until the host
    // clears the halt
    if (c->halt) return;
    c->round = round;
    c->cur = 0;
    c->fcnt[0] = 0;
    c->fcnt[1] = 0;
    c->heavy_cnt = 0;
    c->wide_cnt = 0;
    c->failcnt = 0;
    c->maxmex = -1;
    c->bigw_cnt = 0;
    c->dcnt = c->accepted;  // the previous round's winners (read with this round's snapshot)
    c->accepted = 0;
    c->fsort_all = 1;
    for (int k = 0; k < 3; ++k) c->und_cnt[k] = 0;
    for (int k = 0; k < 9; ++k) c->bcnt[k] = 0;
    c->async_abort[0] = 0;  // the round's asynchronous fold starts un-aborted
}

// bounded attempt with k = 0: only proposers WITH a coloured neighbour fail
// (coloring_optimized.py:159-164); k_propose counted every proposer.
__global__ void __launch_bounds__(GC_BLOCK) k_b_fail0(GDev g, GLists L) {
    DevCtl* c = g.ctl;
    if (c->halt) return;
    __shared__ ull scratch[2 * GC_WAVES_PER_BLOCK];
    const long long cnt = (long long)c->fcnt[c->cur];
    const int* list = L.F[c->cur];
    ull lf = 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += (long long)gridDim.x * blockDim.x) {
        const int v = list[i];
        bool any = false;
        for (long long e = g.rp[v]; e < g.rp[v + 1] && !any; ++e) any = g.c8[g.col[e]] != GC_C8_NONE;
        lf += any ? 1ull : 0ull;
    }
    __syncthreads();
    gc_block_add(&c->failcnt, lf, scratch);
}

// Work lists.  Every pass reads slot i % 3 of three lists -- light admission (UND
// vertices), heavy admission (UND vertices whose remaining range exceeds GC_B_HEAVY: a
// workgroup each) and eviction (admitted vertices whose eviction time is not final) --
// writes slot (i + 1) % 3 and clears the counters of slot (i + 2) % 3 (read by pass i - 1,
// written by pass i + 1): one launch per list kind per pass, no host round trip.
#define GC_B_HEAVY 2048
struct BLists {
    int* l[3][3];  // [kind][slot]
    int* pend;     // nnz ints: each listed light vertex's still-pending entries, at rp[v] (see below)
    int* watch;    // n ints: an undecided vertex's smallest pending entry at its last scan (asynchronous fold)
    const int* nhe;  // n ints: the row's higher-degree earlier entries (gc_prep.hip's class 2)
};
// Row layout (the (deg, pos) rank partition, gc_prep.hip): [lower degree | equal degree and
// earlier | higher degree and earlier | the rest (later positions of equal or higher degree)].
// An arrival of v can only be refused by an earlier u with deg(u) >= deg(v): the admission
// range [nlow[v] - neq[v], nlow[v] + nhe[v]).  v can only be evicted by a later u with
// deg(u) > deg(v): the eviction range [nlow[v] + nhe[v], deg(v)) (its equal-degree entries
// are skipped by their degree).
__device__ __forceinline__ int b_adm_end(const GDev& g, const BLists& B, int v) { return g.nlow[v] + B.nhe[v]; }
// Pending entries (round 4).  A flag that reads 0 is final (a later arrival, a refused or
// other-candidate vertex, an eviction before v), so after its first scan a light vertex only
// ever needs the entries that were still pending: each scan writes them, compacted, to
// pend[rp[v] ...] (in place after the first), and lcur[v] = -(count) - 1 says so.  An admitted
// vertex's eviction scan likewise keeps its not-refused potential evictors there (its
// admission entries are done with); lcur[v] = GC_B_EVCOL until its first eviction scan.
// Heavy admissions (a workgroup each) keep the cursor form, lcur[v] >= 0: the first pending
// entry of the row.  A pass's work is then the pending entries, not the rest of every row.
#define GC_B_EVCOL 0x7FFFFFFF
#define GC_B_PMARK 0x80000000u  // marks an entry read from pend[] (its degree was checked)
__device__ __forceinline__ ull* b_cnt(DevCtl* c, int kind, int slot) { return &c->bcnt[kind * 3 + slot]; }
// a list count at the start of a pass (written by an earlier launch)
__device__ __forceinline__ long long b_count(DevCtl* c, int kind, int slot) { return (long long)*b_cnt(c, kind, slot); }

// gc_chunk_edges_at over per-owner sources: owner o's x-th entry is s_src[o][x]; load(o, u).
// skip(o): the owner needs no more entries (its entries after that point are not read)
struct BNoSkip {
    __device__ bool operator()(int) const { return false; }
};
template <typename Load, typename Apply, typename Skip = BNoSkip>
__device__ __forceinline__ void b_chunk_edges(const int* const* s_src, int excl, int total, Load load, Apply apply,
                                              Skip skip = Skip()) {
    const int lane = gc_lane();
    for (int base = 0; base < total; base += GC_SLOTS * GC_WAVE) {
        int o[GC_SLOTS], x[GC_SLOTS], u[GC_SLOTS];
        bool ok[GC_SLOTS];
#pragma unroll
        for (int k = 0; k < GC_SLOTS; ++k) {
            const int e = base + k * GC_WAVE + lane;
            o[k] = gc_owner(excl, e);
            x[k] = e - __shfl(excl, o[k], GC_WAVE);
            ok[k] = e < total && !skip(o[k]);
        }
#pragma unroll
        for (int k = 0; k < GC_SLOTS; ++k) u[k] = ok[k] ? s_src[o[k]][x[k]] : 0;
        decltype(load(0, 0)) gv[GC_SLOTS];
#pragma unroll
        for (int k = 0; k < GC_SLOTS; ++k) gv[k] = ok[k] ? load(o[k], u[k]) : decltype(load(0, 0)){};
#pragma unroll
        for (int k = 0; k < GC_SLOTS; ++k)
            if (ok[k]) apply(o[k], u[k], gv[k], x[k]);
    }
}

// (Row layout and the two ranges: b_adm_end above.)
// Round start: every proposer is undecided; its admission range starts at the equal-degree
// entries; eviction times unknown (-1).
__global__ void __launch_bounds__(GC_BLOCK) k_b_init(GDev g, GLists L, BLists B, int* ev, const int* neq) {
    DevCtl* c = g.ctl;
    if (c->halt) return;  // a list overflowed (k_b_reset keeps the halt)
    __shared__ int s_stage[GC_WAVES_PER_BLOCK][GC_STAGE_CAP];
    const int w = threadIdx.x / GC_WAVE;
    GcStage st{s_stage[w], 0, g.list_cap, &g.ctl->loop_err, &g.ctl->halt};
    const long long cnt = (long long)c->fcnt[c->cur];
    const int* list = L.F[c->cur];
    const long long steps = (cnt + GC_WAVE - 1) / GC_WAVE;
    for (long long sidx = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w; sidx < steps;
         sidx += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
        const long long i = sidx * GC_WAVE + gc_lane();
        const int v = i < cnt ? list[i] : -1;
        bool heavy = false;
        if (v >= 0) {
            const int bc = g.nlow[v] - neq[v];
            g.lcur[v] = bc;
            ev[v] = -1;
            B.watch[v] = 0;
            heavy = b_adm_end(g, B, v) - bc > GC_B_HEAVY;
        }
        gc_wave_append(heavy, v, B.l[1][0], b_cnt(c, 1, 0));
        gc_stage_push(st, v >= 0 && !heavy, v, B.l[0][0], b_cnt(c, 0, 0));
    }
    gc_stage_flush_block(st, B.l[0][0], b_cnt(c, 0, 0));
}

// eviction pass over list slot i % 3: ev(u) = the smallest not-refused potential evictor
// (v' > u listed by u, same candidate, deg(v') > deg(u)); final once that evictor is
// admitted or there is none (INF), else u stays listed.  Workgroup bid of nblk.
__device__ void b_ev_pass(GDev& g, BLists& B, int* ev, int pass, int bid, int nblk) {
    DevCtl* c = g.ctl;
    const int rs = pass % 3, ws = (pass + 1) % 3, zs = (pass + 2) % 3;
    if (bid == 0 && threadIdx.x < 3) *b_cnt(c, threadIdx.x, zs) = 0ull;
    __shared__ int s_stage[GC_WAVES_PER_BLOCK][GC_STAGE_CAP];
    __shared__ const int* s_src[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int* s_dst[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_np[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_min[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_v[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_d[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ unsigned s_c6[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_cv[GC_WAVES_PER_BLOCK][GC_WAVE];
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    const int* __restrict__ list = B.l[2][rs];
    const long long cnt = b_count(c, 2, rs);
    const unsigned char* __restrict__ k8 = g.k8;
    GcStage st{s_stage[w], 0, g.list_cap, &g.ctl->loop_err, &g.ctl->halt};
    const int vpw = gc_vpw(cnt, (long long)nblk * GC_WAVES_PER_BLOCK);
    const long long nch = gc_nchunks(cnt, vpw);
    for (long long ch = (long long)bid * GC_WAVES_PER_BLOCK + w; ch < nch;
         ch += (long long)nblk * GC_WAVES_PER_BLOCK) {
        const long long idx = ch * vpw + lane;
        const int v = (lane < vpw && idx < cnt) ? list[idx] : -1;
        const unsigned kv = v >= 0 ? (unsigned)k8[v] : 0u;
        const int d = v >= 0 ? g.deg[v] : 0;
        const int lc = v >= 0 ? g.lcur[v] : GC_B_EVCOL;
        const long long r0 = v >= 0 ? g.rp[v] : 0;
        // Watch: after its first scan, ev(v) can only move when the evictor it names is
        // refused -- while that one is undecided v stays listed unscanned, once it is admitted
        // ev(v) is final; only a refusal asks for a rescan of the kept entries.
        int watch = 0;  // 1: still pending, no scan; 2: final, no scan
        if (v >= 0 && lc != GC_B_EVCOL) {
            const unsigned st = gc_k8_state(k8[ev[v]]);
            watch = st == GC_JP_UND ? 1 : (st == GC_JP_IN ? 2 : 0);
        }
        int len = 0;
        if (v >= 0 && lc == GC_B_EVCOL) {  // first eviction scan: the row's eviction range
            const int lo = b_adm_end(g, B, v);
            len = d - lo;
            s_src[w][lane] = g.col + r0 + lo;
        } else if (v >= 0 && watch == 0) {  // the kept potential evictors
            len = -lc - 1;
            s_src[w][lane] = B.pend + r0;
        }
        s_dst[w][lane] = B.pend + r0;
        s_np[w][lane] = 0;
        s_min[w][lane] = GC_B_INF;
        s_v[w][lane] = v;
        s_d[w][lane] = d;
        s_c6[w][lane] = v >= 0 ? gc_k8_cand(kv) : 0x100u;
        s_cv[w][lane] = v >= 0 ? b_cand(g, v, kv) : -1;
        const int incl = gc_wave_incl_scan(len);
        const int excl = incl - len;
        const int total = __shfl(incl, GC_WAVE - 1, GC_WAVE);
        gc_wave_sync();
        // a kept entry (marked) passed the static tests (later arrival, higher degree, same
        // candidate): only its state can change
        b_chunk_edges(
            s_src[w], excl, total,
            [&](int, int um) {
                const int u = um & 0x7FFFFFFF;
                return ((unsigned)um & GC_B_PMARK) ? (ull)k8[u] : ((ull)(unsigned)g.deg[u] << 32) | (ull)k8[u];
            },
            [&](int o, int um, ull du, int) {
                const int u = um & 0x7FFFFFFF;
                const unsigned ku = (unsigned)du & 0xFFu;
                if (gc_k8_state(ku) == GC_JP_OUT) return;
                if (!((unsigned)um & GC_B_PMARK)) {
                    if (u <= s_v[w][o] || (int)(du >> 32) <= s_d[w][o]) return;
                    if (!b_same(g, u, ku, s_c6[w][o], s_cv[w][o])) return;
                }
                atomicMin(&s_min[w][o], u);
                s_dst[w][o][atomicAdd(&s_np[w][o], 1)] = (int)((unsigned)u | GC_B_PMARK);
            });
        gc_wave_sync();
        bool pend = watch == 1;
        if (v >= 0 && watch == 0) {
            const int e = s_min[w][lane];
            ev[v] = e;
            pend = e != GC_B_INF && gc_k8_state(k8[e]) != GC_JP_IN;
            if (pend) g.lcur[v] = -s_np[w][lane] - 1;
        }
        gc_stage_push(st, pend, v, B.l[2][ws], b_cnt(c, 2, ws));
    }
    gc_stage_flush_block(st, B.l[2][ws], b_cnt(c, 2, ws));
}

__global__ void __launch_bounds__(GC_BLOCK) k_b_ev(GDev g, BLists B, int* ev, int pass) {
    if (g.ctl->halt) return;
    b_ev_pass(g, B, ev, pass, blockIdx.x, gridDim.x);
}

// admission flag of one entry u for v (vo): 1 = u admitted and still present at v's
// arrival (v refused), 2 = not known yet, 0 = never matters again.  Entries in the range
// all have deg(u) >= deg(v) (row layout above).
__device__ __forceinline__ unsigned b_adm_flag(const GDev& g, int vo, int u, unsigned ku, unsigned c6, int cv,
                                               const int* ev) {
    if (u >= vo) return 0u;  // later arrivals (and self-loops) never count
    const unsigned st = gc_k8_state(ku);
    if (st == GC_JP_OUT || !b_same(g, u, ku, c6, cv)) return 0u;
    if (st != GC_JP_IN) return 2u;
    const int e = ev[u];
    if (e > vo) return 1u;                                   // still admitted at v's arrival
    if (e >= 0 && gc_k8_state(g.k8[e]) == GC_JP_IN) return 0u;  // evicted before v
    return 2u;                                               // eviction time not known yet
}

// decision of v after a scan: OUT / IN (listed for its eviction time) / still undecided
// (resumes at its first pending entry; light or heavy list by the range left)
__device__ __forceinline__ void b_adm_decide(GDev& g, BLists& B, DevCtl* c, int ws, int v, unsigned kv, unsigned f,
                                             int first, int* dst_kind) {
    *dst_kind = -1;
    if (f & 1u) {
        g.k8[v] = (unsigned char)((kv & ~3u) | GC_JP_OUT);
    } else if (f & 2u) {
        const int bc = g.lcur[v] + first;
        g.lcur[v] = bc;
        *dst_kind = b_adm_end(g, B, v) - bc > GC_B_HEAVY ? 1 : 0;
    } else {
        g.k8[v] = (unsigned char)((kv & ~3u) | GC_JP_IN);
        g.lcur[v] = GC_B_EVCOL;
        *dst_kind = 2;
    }
}

// admission of the heavy list, slot i % 3: a workgroup per vertex (k_b_adm's workgroups,
// before their light chunks)
__device__ void b_adm_heavy(GDev& g, BLists& B, const int* ev, int pass, int bid, int nblk) {
    DevCtl* c = g.ctl;
    const int rs = pass % 3, ws = (pass + 1) % 3;
    const long long cnt = b_count(c, 1, rs);
    if (cnt == 0) return;
    __shared__ unsigned s_flag;
    __shared__ int s_first;
    const int* list = B.l[1][rs];
    for (long long i = bid; i < cnt; i += nblk) {
        const int v = list[i];
        const unsigned kv = g.k8[v];
        const unsigned c6 = gc_k8_cand(kv);
        const int cv = b_cand(g, v, kv);
        const int bc = g.lcur[v];
        const long long s0 = g.rp[v] + bc, s1 = g.rp[v] + b_adm_end(g, B, v);
        if (threadIdx.x == 0) {
            s_flag = 0u;
            s_first = 0x7FFFFFFF;
        }
        __syncthreads();
        for (long long e0 = s0; e0 < s1; e0 += GC_SLOTS * (long long)blockDim.x) {
            int u[GC_SLOTS];
            unsigned ku[GC_SLOTS];
#pragma unroll
            for (int k = 0; k < GC_SLOTS; ++k) {
                const long long e = e0 + (long long)k * blockDim.x + threadIdx.x;
                u[k] = e < s1 ? g.col[e] : -1;
            }
#pragma unroll
            for (int k = 0; k < GC_SLOTS; ++k) ku[k] = u[k] >= 0 ? (unsigned)g.k8[u[k]] : 0u;
#pragma unroll
            for (int k = 0; k < GC_SLOTS; ++k) {
                if (u[k] < 0) continue;
                const unsigned f = b_adm_flag(g, v, u[k], ku[k], c6, cv, ev);
                if (f) atomicOr(&s_flag, f);
                if (f == 2u) atomicMin(&s_first, (int)(e0 + (long long)k * blockDim.x + threadIdx.x - s0));
            }
            __syncthreads();
            const bool refused = (s_flag & 1u) != 0;  // refused: the rest cannot change it
            __syncthreads();
            if (refused) break;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int kind = -1;
            b_adm_decide(g, B, c, ws, v, kv, s_flag, s_first, &kind);
            if (kind >= 0) B.l[kind][ws][atomicAdd(b_cnt(c, kind, ws), 1ull)] = v;
        }
        __syncthreads();
    }
}

// admission pass, slot i % 3: the heavy list (a workgroup per vertex), then the light list
// (wave chunks)
__device__ void b_adm_pass(GDev& g, BLists& B, const int* ev, int pass, int bid, int nblk) {
    b_adm_heavy(g, B, ev, pass, bid, nblk);
    DevCtl* c = g.ctl;
    const int rs = pass % 3, ws = (pass + 1) % 3;
    __shared__ int s_stage[GC_WAVES_PER_BLOCK][GC_STAGE_CAP];
    __shared__ int s_estage[GC_WAVES_PER_BLOCK][GC_STAGE_CAP];
    __shared__ const int* s_src[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int* s_dst[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ unsigned s_flag[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_np[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_v[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ unsigned s_c6[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_cv[GC_WAVES_PER_BLOCK][GC_WAVE];
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    const int* __restrict__ list = B.l[0][rs];
    const long long cnt = b_count(c, 0, rs);
    const unsigned char* __restrict__ k8 = g.k8;
    GcStage st{s_stage[w], 0, g.list_cap, &g.ctl->loop_err, &g.ctl->halt}, est{s_estage[w], 0, g.list_cap, &g.ctl->loop_err, &g.ctl->halt};
    const int vpw = gc_vpw(cnt, (long long)nblk * GC_WAVES_PER_BLOCK);
    const long long nch = gc_nchunks(cnt, vpw);
    for (long long ch = (long long)bid * GC_WAVES_PER_BLOCK + w; ch < nch;
         ch += (long long)nblk * GC_WAVES_PER_BLOCK) {
        const long long idx = ch * vpw + lane;
        const int v = (lane < vpw && idx < cnt) ? list[idx] : -1;
        const unsigned kv = v >= 0 ? (unsigned)k8[v] : 0u;
        const int lc = v >= 0 ? g.lcur[v] : 0;
        const long long r0 = v >= 0 ? g.rp[v] : 0;
        int len = 0;
        if (v >= 0 && lc >= 0) {  // first light scan: the row from the cursor
            len = b_adm_end(g, B, v) - lc;
            s_src[w][lane] = g.col + r0 + lc;
        } else if (v >= 0) {  // the still-pending entries
            len = -lc - 1;
            s_src[w][lane] = B.pend + r0;
        }
        s_dst[w][lane] = B.pend + r0;
        s_flag[w][lane] = 0;
        s_np[w][lane] = 0;
        s_v[w][lane] = v;
        s_c6[w][lane] = v >= 0 ? gc_k8_cand(kv) : 0x100u;
        s_cv[w][lane] = v >= 0 ? b_cand(g, v, kv) : -1;
        const int incl = gc_wave_incl_scan(len);
        const int excl = incl - len;
        const int total = __shfl(incl, GC_WAVE - 1, GC_WAVE);
        gc_wave_sync();
        b_chunk_edges(
            s_src[w], excl, total, [&](int, int u) { return (unsigned)k8[u]; },
            [&](int o, int u, unsigned ku, int) {
                const unsigned f = b_adm_flag(g, s_v[w][o], u, ku, s_c6[w][o], s_cv[w][o], ev);
                if (f) atomicOr(&s_flag[w][o], f);
                if (f == 2u) s_dst[w][o][atomicAdd(&s_np[w][o], 1)] = u;
            });
        gc_wave_sync();
        int kind = -1;
        if (v >= 0) {
            const unsigned f = s_flag[w][lane];
            if (f & 1u) {
                g.k8[v] = (unsigned char)((kv & ~3u) | GC_JP_OUT);
            } else if (f & 2u) {
                g.lcur[v] = -s_np[w][lane] - 1;
                B.watch[v] = 0;  // the compacted list from its start (the asynchronous fold's cursor)
                kind = 0;
            } else {
                g.k8[v] = (unsigned char)((kv & ~3u) | GC_JP_IN);
                g.lcur[v] = GC_B_EVCOL;
                kind = 2;
            }
        }
        gc_wave_append(kind == 1, v, B.l[1][ws], b_cnt(c, 1, ws));
        gc_stage_push(st, kind == 0, v, B.l[0][ws], b_cnt(c, 0, ws));
        gc_stage_push(est, kind == 2, v, B.l[2][ws], b_cnt(c, 2, ws));
    }
    gc_stage_flush_block(st, B.l[0][ws], b_cnt(c, 0, ws));
    gc_stage_flush_block(est, B.l[2][ws], b_cnt(c, 2, ws));
}

__global__ void __launch_bounds__(GC_BLOCK) k_b_adm(GDev g, BLists B, const int* ev, int pass) {
    if (g.ctl->halt) return;
    b_adm_pass(g, B, ev, pass, blockIdx.x, gridDim.x);
}

// (Round 4 measured a pass's eviction and admission halves in ONE launch, no grid barrier
// between them: R-MAT-24 656 -> 1000 ms, uniform 10M 20.7 -> 24.7 ms, profiles/r04/i; removed.)

// (Round 4 also ran the fold's deep end in ONE workgroup, passes a workgroup barrier apart,
// while the lists stayed small (k_b_tail): R-MAT-24 slower at every cap tried -- 2048 light /
// 4 heavy / 4096 evictions 656 -> 723 ms, 256/0/512 658 -> 677, 64/0/128 658 -> 661,
// profiles/r04/h, r04/j; removed.)


// winners: admitted and never evicted, coloured (coloring_optimized.py:129-140); with hub
// bitmaps, pushed into the hubs listing them (gc_hub_push_wave)
// check_ws >= 0 (pipelined rounds: the host enqueued this commit without waiting for the
// fold): the round's own decisions, as the host makes them otherwise -- no uncoloured vertex
// left: GC_H_DONE; a bounded attempt with a failing proposer: GC_H_FAILED (nothing committed,
// the state at the round start stays); the fold's lists of slot check_ws not empty (a give-up
// of the asynchronous fold, or more passes needed): GC_H_SWEEPS.  Every workgroup reaches the
// same decision from words no kernel of this launch writes.
__global__ void __launch_bounds__(GC_BLOCK) k_b_commit(GDev g, GLists L, const int* ev, int* big, int check_ws) {
    DevCtl* c = g.ctl;
    if (c->halt) return;
    if (check_ws >= 0) {
        int h = GC_RUN;
        if (c->fcnt[c->cur] == 0) h = GC_H_DONE;
        else if (c->kbound >= 0 && c->failcnt > 0) h = GC_H_FAILED;
        else if (c->loop_err) h = GC_H_STALLED;
        else if (c->bcnt[check_ws] + c->bcnt[3 + check_ws] + c->bcnt[6 + check_ws]) h = GC_H_SWEEPS;
        if (h != GC_RUN) {
            if (blockIdx.x == 0 && threadIdx.x == 0) c->halt = h;
            return;
        }
    }
    __shared__ ull scratch[2 * GC_WAVES_PER_BLOCK];
    __shared__ long long s_start[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_cc[GC_WAVES_PER_BLOCK][GC_WAVE];
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    const long long cnt = (long long)c->fcnt[c->cur];
    const int* list = L.F[c->cur];
    const int round = (int)(c->round + 1);
    const bool want_cround = c->want_cround != 0;
    long long lmaxc = -1;
    ull lacc = 0, lsum = 0;
    const long long steps = (cnt + GC_WAVE - 1) / GC_WAVE;
    for (long long sidx = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w; sidx < steps;
         sidx += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
        const long long i = sidx * GC_WAVE + lane;
        const int v = i < cnt ? list[i] : -1;
        const unsigned kv = v >= 0 ? (unsigned)g.k8[v] : 0u;
        const bool win = v >= 0 && gc_k8_state(kv) == GC_JP_IN && ev[v] == GC_B_INF;
        int cc = 0;
        if (win) {
            cc = b_cand(g, v, kv);
            gc_commit_colour(g, v, cc);
            if (want_cround) g.cround[v] = round;
            lmaxc = cc > lmaxc ? cc : lmaxc;
            lacc++;
            lsum += (ull)g.deg[v];
        }
        if (g.hbits_w) gc_hub_push_wave(g, win, v, cc, s_start[w], s_cc[w], big, &c->bigw_cnt);  // wave-uniform
    }
    __syncthreads();
    gc_block_max(&c->maxcolor, lmaxc, (long long*)scratch);
    gc_block_add(&c->accepted, lacc, scratch);
    gc_stat_add(g, GC_K_COMMIT, lsum, lacc, scratch);
}

// (Round 3's asynchronous fold -- the round's passes in one launch on a resident grid,
// GC_B_ASYNC=1 -- measured R-MAT-24 855.6 -> 1036.9 ms in round 4, profiles/r04/c: removed.)

// ------------------------------------------------------------------------------------
// Asynchronous fold (round 4, GC_B_ASYNC): after the host's first full-grid passes (the
// bandwidth-bound first scans, which leave every light vertex's pending entries compacted),
// the rest of the round's fold in ONE launch on a resident grid, with no host round trip and
// no launch per pass.  Every wave owns a static slice of the round's items -- light
// admissions and eviction times (edge-balanced wave chunks over their pending / kept
// entries, as k_b_adm / k_b_ev) and heavy admissions (a wave each, a resumable scan that
// stops at the first refusing or undecided entry) -- and passes over its unsettled items
// until none is left; an admitted vertex becomes an eviction item of the same wave.  Every
// decision is monotone (UND -> IN / OUT; eviction times only grow and are final once the
// evictor named is admitted or there is none) and the earliest unsettled item in arrival
// order can always settle, so the waves converge without waiting on each other.  States
// and eviction times other waves read are stored and loaded agent-scope (sc1); a vertex's
// cursor, pending entries and own byte are only ever touched by its own wave.  A wave past
// the budget hands its unsettled items to the pass lists of the next slot and the host's
// passes finish them.  (Round 3's asynchronous fold ran from the round's first pass,
// rescanning whole rows: 21% slower than the passes, removed in round 4.)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ bool b_async_stop(DevCtl* c, ull t0, long long budget) {
    int stop = 0;
    if (gc_lane() == 0) {
        stop = __hip_atomic_load(&c->async_abort[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!stop && (long long)(wall_clock64() - t0) > budget) {
            stop = 1;
            if (atomicCAS(&c->async_abort[0], 0, 1) == 0) atomicAdd(&c->async_aborts, 1ull);
        }
    }
    return __shfl(stop, 0, GC_WAVE) != 0;
}

#ifdef GC_B_PROF
// (diagnostic build, -DGC_B_PROF: per round, the fold's slowest wave and its work; read by
// gc_b_prof_dump at the end of the colouring, GC_B_PROF_OUT=path)
#define GC_B_PROF_ROUNDS 4096
#define GC_B_PROF_K 12
__device__ ull gc_bprof[GC_B_PROF_ROUNDS][GC_B_PROF_K];
#endif

// a work item is v | kind << GC_BI_SHIFT (kind 0 admission, 2 eviction time): non-negative
// for n < 2^29 (-1 marks an empty lane), so the host runs k_b_async only below that
#define GC_BI_SHIFT 29
#define GC_BI_MASK ((1 << GC_BI_SHIFT) - 1)

// b_adm_flag with agent-scope loads of the states and eviction times other waves write
__device__ __forceinline__ unsigned b_adm_flag_a(const GDev& g, int vo, int u, unsigned ku, unsigned c6, int cv,
                                                 const int* ev) {
    if (u >= vo) return 0u;
    const unsigned st = gc_k8_state(ku);
    if (st == GC_JP_OUT || !b_same(g, u, ku, c6, cv)) return 0u;
    if (st != GC_JP_IN) return 2u;
    const int e = gc_aldi(ev + u);
    if (e > vo) return 1u;
    if (e >= 0 && gc_k8_state(gc_ald8(g.k8 + e)) == GC_JP_IN) return 0u;
    return 2u;
}

struct BAsyncLds {  // one wave's rows
    const int* src[GC_WAVE];
    int* dst[GC_WAVE];
    unsigned flag[GC_WAVE];
    int np[GC_WAVE];
    int minv[GC_WAVE];
    int v[GC_WAVE];
    int d[GC_WAVE];
    unsigned c6[GC_WAVE];
    int cv[GC_WAVE];
    int kind[GC_WAVE];
};

// one pass over the wave's light admission / eviction items l1[0, n1); the unsettled ones
// are compacted to the front (an admitted vertex comes back as an eviction item); returns
// their number
// Admission cursors (g.b_watch = R > 0, 4): between full rescans (every R-th pass of the wave) an
// admission item reads only a window of g.b_awin (8) of its pending entries from a cursor
// (B.watch[v]: the entries before it are settled 0), advances the cursor past the settled
// prefix and stops at the first entry still pending; a refusal in the window settles it, the
// cursor reaching the end admits it.  Each pending entry is then read about once more after it
// settles, where a rescan of every pending entry per settled one cost O(pending^2) (round 5:
// 5.8 of the fold's 10.7 G entries were admission rescans on R-MAT-24).  A refusal by an entry
// past the first pending one is seen at the next full rescan at the latest; the decisions are
// the same.
__device__ int b_async_chunk_pass(GDev& g, const BLists& B, int* l1, int n1, int* ev, BAsyncLds& s, ull* scanned,
                                  ull npass) {
    const bool full_pass = g.b_watch <= 0 || npass % (ull)g.b_watch == 0;
    const int lane = gc_lane();
    int nw = 0;
    for (int c0 = 0; c0 < n1; c0 += GC_WAVE) {
        const int it = c0 + lane < n1 ? l1[c0 + lane] : -1;
        const int v = it >= 0 ? (it & GC_BI_MASK) : -1;
        const int kind = it >= 0 ? (it >> GC_BI_SHIFT) : -1;
        const unsigned kv = v >= 0 ? (unsigned)g.k8[v] : 0u;  // its candidate (fixed for the round)
        const int d = v >= 0 ? g.deg[v] : 0;
        const int lc = v >= 0 ? g.lcur[v] : 0;
        const long long r0 = v >= 0 ? g.rp[v] : 0;
        int watch = 0;  // eviction items: 1 still pending, 2 final, no scan (b_ev_pass)
        if (kind == 2 && lc != GC_B_EVCOL) {
            const unsigned st = gc_k8_state(gc_ald8(g.k8 + ev[v]));
            watch = st == GC_JP_UND ? 1 : (st == GC_JP_IN ? 2 : 0);
        }
        // admission items in the pending-list form: cursor and pending count
        const int anp = (kind == 0 && lc < 0) ? -lc - 1 : 0;
        int acur = 0;
        if (kind == 0 && lc < 0 && g.b_watch > 0) {
            acur = B.watch[v];
            acur = acur < 0 ? 0 : (acur > anp ? anp : acur);
        }
        const bool win = kind == 0 && lc < 0 && !full_pass;  // a window from the cursor
        int len = 0;
        if (win) {
            len = anp - acur < g.b_awin ? anp - acur : g.b_awin;
            s.src[lane] = B.pend + r0 + acur;
        } else if (kind == 0) {
            len = lc >= 0 ? b_adm_end(g, B, v) - lc : anp - acur;
            s.src[lane] = lc >= 0 ? g.col + r0 + lc : B.pend + r0 + acur;
        } else if (kind == 2 && lc == GC_B_EVCOL) {
            const int lo = b_adm_end(g, B, v);
            len = d - lo;
            s.src[lane] = g.col + r0 + lo;
        } else if (kind == 2 && watch == 0) {
            len = -lc - 1;
            s.src[lane] = B.pend + r0;
        }
        s.dst[lane] = B.pend + r0;
        s.flag[lane] = 0;
        s.np[lane] = 0;
        s.minv[lane] = GC_B_INF;
        s.v[lane] = v;
        s.d[lane] = d;
        s.c6[lane] = v >= 0 ? gc_k8_cand(kv) : 0x100u;
        s.cv[lane] = v >= 0 ? b_cand(g, v, kv) : -1;
        s.kind[lane] = win ? 1 : kind;  // (1: an admission window; no heavy item is listed here)
        const int incl = gc_wave_incl_scan(len);
        const int excl = incl - len;
        const int total = __shfl(incl, GC_WAVE - 1, GC_WAVE);
        *scanned += (ull)total;
        gc_wave_sync();
        b_chunk_edges(
            s.src, excl, total,
            [&](int o, int um) {
                const int u = um & 0x7FFFFFFF;
                const ull k = (ull)gc_ald8(g.k8 + u);
                return (s.kind[o] == 2 && !((unsigned)um & GC_B_PMARK)) ? ((ull)(unsigned)g.deg[u] << 32) | k : k;
            },
            [&](int o, int um, ull du, int x) {
                const int u = um & 0x7FFFFFFF;
                const unsigned ku = (unsigned)du & 0xFFu;
                if (s.kind[o] == 1) {  // admission window: the first entry still pending
                    const unsigned f = b_adm_flag_a(g, s.v[o], u, ku, s.c6[o], s.cv[o], ev);
                    if (f) atomicOr(&s.flag[o], f);
                    if (f == 2u) atomicMin(&s.minv[o], x);
                } else if (s.kind[o] == 0) {  // admission (k_b_adm)
                    const unsigned f = b_adm_flag_a(g, s.v[o], u, ku, s.c6[o], s.cv[o], ev);
                    if (f) atomicOr(&s.flag[o], f);
                    if (f == 2u) s.dst[o][atomicAdd(&s.np[o], 1)] = u;
                } else {  // eviction time (k_b_ev)
                    if (gc_k8_state(ku) == GC_JP_OUT) return;
                    if (!((unsigned)um & GC_B_PMARK)) {
                        if (u <= s.v[o] || (int)(du >> 32) <= s.d[o]) return;
                        if (!b_same(g, u, ku, s.c6[o], s.cv[o])) return;
                    }
                    atomicMin(&s.minv[o], u);
                    s.dst[o][atomicAdd(&s.np[o], 1)] = (int)((unsigned)u | GC_B_PMARK);
                }
            },
            [&](int o) { return g.b_refskip && s.kind[o] <= 1 && (s.flag[o] & 1u); });  // refused: the rest cannot matter
        gc_wave_sync();
        int keep = -1;  // the item that stays (-1: settled)
        if (win) {
            const unsigned f = s.flag[lane];
            const int x = s.minv[lane];
            if (f & 1u) {
                gc_ast8(g.k8 + v, (kv & ~3u) | GC_JP_OUT);
            } else if (x != GC_B_INF || acur + len < anp) {  // still pending: past the settled prefix
                B.watch[v] = acur + (x != GC_B_INF ? x : len);
                keep = it;
            } else {  // every pending entry settled 0
                g.lcur[v] = GC_B_EVCOL;
                gc_ast8(g.k8 + v, (kv & ~3u) | GC_JP_IN);
                keep = v | (2 << GC_BI_SHIFT);
            }
        } else if (kind == 0) {
            const unsigned f = s.flag[lane];
            if (f & 1u) {
                gc_ast8(g.k8 + v, (kv & ~3u) | GC_JP_OUT);
            } else if (f & 2u) {
                g.lcur[v] = -s.np[lane] - 1;
                if (g.b_watch > 0) B.watch[v] = 0;  // the compacted list from its start
                keep = it;
            } else {
                g.lcur[v] = GC_B_EVCOL;
                gc_ast8(g.k8 + v, (kv & ~3u) | GC_JP_IN);
                keep = v | (2 << GC_BI_SHIFT);  // admitted: its eviction time next
            }
        } else if (kind == 2) {
            if (watch == 1) {
                keep = it;
            } else if (watch == 0) {
                const int e = s.minv[lane];
                gc_asti(ev + v, e);
                if (e != GC_B_INF && gc_k8_state(gc_ald8(g.k8 + e)) != GC_JP_IN) {
                    g.lcur[v] = -s.np[lane] - 1;
                    keep = it;
                }
            }
        }
        const ull km = __ballot(keep >= 0);
        if (keep >= 0) l1[nw + __popcll(km & gc_lanemask_lt())] = keep;
        nw += __popcll(km);
        gc_wave_sync();
    }
    return nw;
}

// one pass over the wave's heavy admissions l2[0, n2), one vertex at a time (the wave's
// lanes over its row from the cursor, GC_HUB_UNR entries each in flight): a refusing entry
// settles it OUT, the first undecided entry is its new cursor, the end of the row admits it
// (appended to l1 as an eviction item at *n1).  Returns the heavy items left.
__device__ int b_async_heavy_pass(GDev& g, const BLists& B, int* l2, int n2, int* l1, int* n1, int* ev, ull* scanned) {
    const int lane = gc_lane();
    int nw = 0;
    for (int i = 0; i < n2; ++i) {
        const int v = l2[i];
        const unsigned kv = g.k8[v];
        const unsigned c6 = gc_k8_cand(kv);
        const int cv = b_cand(g, v, kv);
        const int d = b_adm_end(g, B, v);  // the admission range's end
        const long long base = g.rp[v];
        int pos = g.lcur[v];
        bool refused = false;
        int pend = -1;
        while (pos < d && !refused && pend < 0) {
            int u[GC_HUB_UNR];
            unsigned f[GC_HUB_UNR];
#pragma unroll
            for (int k = 0; k < GC_HUB_UNR; ++k) {
                const int e = pos + k * GC_WAVE + lane;
                u[k] = e < d ? g.col[base + e] : -1;
            }
#pragma unroll
            for (int k = 0; k < GC_HUB_UNR; ++k)
                f[k] = u[k] >= 0 ? b_adm_flag_a(g, v, u[k], gc_ald8(g.k8 + u[k]), c6, cv, ev) : 0u;
#pragma unroll
            for (int k = 0; k < GC_HUB_UNR; ++k) {
                if (__ballot(f[k] == 1u)) refused = true;
                const ull mb = __ballot(f[k] == 2u);
                if (mb && pend < 0) pend = pos + k * GC_WAVE + __builtin_ctzll(mb);
            }
            pos += GC_HUB_UNR * GC_WAVE;
            *scanned += GC_HUB_UNR * GC_WAVE;
        }
        if (refused) {
            if (lane == 0) gc_ast8(g.k8 + v, (kv & ~3u) | GC_JP_OUT);
        } else if (pend >= 0) {
            if (lane == 0) {
                g.lcur[v] = pend;
                l2[nw] = v;
            }
            ++nw;
        } else {
            if (lane == 0) {
                g.lcur[v] = GC_B_EVCOL;
                gc_ast8(g.k8 + v, (kv & ~3u) | GC_JP_IN);
                l1[*n1] = v | (2 << GC_BI_SHIFT);
            }
            ++*n1;
        }
        gc_wave_sync();
    }
    return nw;
}

// Resident form of a wave's fold, once its unsettled items fit one chunk (at most 64 light
// items, no heavy one) and their entries fit the wave's LDS (GC_B_RES_CAP): each lane keeps its
// item's words in registers and its pending (admission) or kept (eviction) entries in LDS, so
// a pass is the entries' state gathers alone (k8[u]; ev[u] and k8[ev[u]] for an admitted u) --
// a chunk pass first re-reads the list, the item's words and the entries from memory, and in
// the deep rounds every hop of the fold's dependency chain waits for one such pass
// (profiles/r05/o: ~4.5 us a pass, 100-300 passes a round).  The decisions are b_async_chunk_pass's.
// Region of a lane: max(its entries now, the eviction range it may need once admitted).  The
// stop check runs only on a pass without progress.  Returns -1 (not eligible: nothing
// changed), 0 (every item settled) or the items left on a stop, written back in the global
// form (l1, lcur, pend) for the hand-off.
#ifndef GC_B_RES_CAP  // 768: the fold's LDS allows 6 workgroups per CU (1536: 4, 1024: 5; profiles/r05/at, av)
#define GC_B_RES_CAP 768
#endif
__device__ int b_async_resident(GDev& g, const BLists& B, int* l1, int n1, int* ev, BAsyncLds& s, int* pe, DevCtl* c,
                                ull t0, long long budget, bool* stop, ull* npass, ull* scanned) {
    const int lane = gc_lane();
    const int it0 = lane < n1 ? l1[lane] : -1;
    int v = it0 >= 0 ? (it0 & GC_BI_MASK) : -1;
    int kind = it0 >= 0 ? (it0 >> GC_BI_SHIFT) : -1;
    unsigned kv = v >= 0 ? (unsigned)g.k8[v] : 0u;  // own byte: only this wave writes it
    const int d = v >= 0 ? g.deg[v] : 0;
    const int lo = v >= 0 ? b_adm_end(g, B, v) : 0;  // the eviction range's start
    const int lc = v >= 0 ? g.lcur[v] : 0;
    const long long r0 = v >= 0 ? g.rp[v] : 0;
    bool evcol = kind == 2 && lc == GC_B_EVCOL;
    int np = (v >= 0 && !evcol) ? -lc - 1 : 0;
    int evv = (kind == 2 && !evcol) ? ev[v] : -1;  // own eviction time (only this wave writes it)
    const bool bad = kind == 0 && lc >= 0;          // first admission scan not done
    const int need = kind == 0 ? max(np, d - lo) : (evcol ? d - lo : np);
    const int incl = gc_wave_incl_scan(need);
    const int off = incl - need;
    if (__ballot(bad) || __shfl(incl, GC_WAVE - 1, GC_WAVE) > GC_B_RES_CAP) return -1;
    // the entries into LDS (flat over the wave's lanes)
    {
        const int pin = gc_wave_incl_scan(np);
        const int pex = pin - np;
        const int ptot = __shfl(pin, GC_WAVE - 1, GC_WAVE);
        s.src[lane] = B.pend + r0;
        s.np[lane] = off;
        gc_wave_sync();
        for (int b0 = 0; b0 < ptot; b0 += GC_WAVE) {  // every lane runs gc_owner
            const int e = b0 + lane;
            const int o = gc_owner(pex, e < ptot ? e : 0);
            const int x = e - __shfl(pex, o, GC_WAVE);
            if (e < ptot) pe[s.np[o] + x] = s.src[o][x];
        }
        gc_wave_sync();
    }
    const unsigned c6 = v >= 0 ? gc_k8_cand(kv) : 0x100u;
    const int cv = v >= 0 ? b_cand(g, v, kv) : -1;
    int n = __popcll(__ballot(v >= 0));
    int idle = 0;
    int acur = 0;  // admission items: the cursor into their pending entries (b_async_chunk_pass)
    if (kind == 0 && g.b_watch > 0) {
        acur = B.watch[v];
        acur = acur < 0 ? 0 : (acur > np ? np : acur);
    }
    while (n > 0) {
        ++*npass;
        const bool win = kind == 0 && g.b_watch > 0 && *npass % (ull)g.b_watch != 0;
        int watch = 0;  // eviction items: 1 still pending, 2 final, no scan
        if (kind == 2 && !evcol) {
            const unsigned st = gc_k8_state(gc_ald8(g.k8 + evv));
            watch = st == GC_JP_UND ? 1 : (st == GC_JP_IN ? 2 : 0);
        }
        int len = 0;
        if (win) {
            len = np - acur < g.b_awin ? np - acur : g.b_awin;
            s.src[lane] = pe + off + acur;
        } else if (kind == 0) {
            len = np - acur;
            s.src[lane] = pe + off + acur;
        } else if (kind == 2 && !evcol && watch == 0) {
            len = np;
            s.src[lane] = pe + off;
        } else if (kind == 2 && evcol) {
            len = d - lo;
            s.src[lane] = g.col + r0 + lo;
        }
        s.dst[lane] = pe + off;
        s.flag[lane] = 0;
        s.np[lane] = 0;
        s.minv[lane] = GC_B_INF;
        s.v[lane] = v;
        s.d[lane] = d;
        s.c6[lane] = c6;
        s.cv[lane] = cv;
        s.kind[lane] = win ? 1 : kind;
        const int li = gc_wave_incl_scan(len);
        const int le = li - len;
        const int total = __shfl(li, GC_WAVE - 1, GC_WAVE);
        *scanned += (ull)total;
        gc_wave_sync();
        b_chunk_edges(
            s.src, le, total,
            [&](int o, int um) {
                const int u = um & 0x7FFFFFFF;
                const ull k = (ull)gc_ald8(g.k8 + u);
                return (s.kind[o] == 2 && !((unsigned)um & GC_B_PMARK)) ? ((ull)(unsigned)g.deg[u] << 32) | k : k;
            },
            [&](int o, int um, ull du, int x) {
                const int u = um & 0x7FFFFFFF;
                const unsigned ku = (unsigned)du & 0xFFu;
                if (s.kind[o] == 1) {  // admission window
                    const unsigned f = b_adm_flag_a(g, s.v[o], u, ku, s.c6[o], s.cv[o], ev);
                    if (f) atomicOr(&s.flag[o], f);
                    if (f == 2u) atomicMin(&s.minv[o], x);
                } else if (s.kind[o] == 0) {
                    const unsigned f = b_adm_flag_a(g, s.v[o], u, ku, s.c6[o], s.cv[o], ev);
                    if (f) atomicOr(&s.flag[o], f);
                    if (f == 2u) s.dst[o][atomicAdd(&s.np[o], 1)] = u;
                } else {
                    if (gc_k8_state(ku) == GC_JP_OUT) return;
                    if (!((unsigned)um & GC_B_PMARK)) {
                        if (u <= s.v[o] || (int)(du >> 32) <= s.d[o]) return;
                        if (!b_same(g, u, ku, s.c6[o], s.cv[o])) return;
                    }
                    atomicMin(&s.minv[o], u);
                    s.dst[o][atomicAdd(&s.np[o], 1)] = (int)((unsigned)u | GC_B_PMARK);
                }
            },
            [&](int o) { return g.b_refskip && s.kind[o] <= 1 && (s.flag[o] & 1u); });  // refused: the rest cannot matter
        gc_wave_sync();
        bool keep = false;
        const unsigned af = s.flag[lane];
        const int ax = s.minv[lane];
        const bool apend = kind == 0 && !(af & 1u) && (win ? (ax != GC_B_INF || acur + len < np) : (af & 2u) != 0);
        if (kind == 0 && apend) {
            if (win) {
                acur += ax != GC_B_INF ? ax : len;
            } else {
                np = s.np[lane];
                acur = 0;
            }
            keep = true;
        } else if (kind == 0) {
            if (af & 1u) {
                gc_ast8(g.k8 + v, (kv & ~3u) | GC_JP_OUT);
            } else {  // admitted: its eviction time next (the row's higher-rank part first)
                kv = (kv & ~3u) | GC_JP_IN;
                gc_ast8(g.k8 + v, kv);
                kind = 2;
                evcol = true;
                np = 0;
                keep = true;
            }
        } else if (kind == 2) {
            if (watch == 1) {
                keep = true;
            } else if (watch == 0) {
                const int e = s.minv[lane];
                gc_asti(ev + v, e);
                evv = e;
                evcol = false;
                np = s.np[lane];
                keep = e != GC_B_INF && gc_k8_state(gc_ald8(g.k8 + e)) != GC_JP_IN;
            }
        }
        if (!keep) {
            v = -1;
            kind = -1;
        }
        const int nn = __popcll(__ballot(keep));
        gc_wave_sync();
        if (nn == 0) return 0;
        if (nn == n) {
            if ((*stop = b_async_stop(c, t0, budget))) {
                n = nn;
                break;
            }
            if (++idle > 2) __builtin_amdgcn_s_sleep(2);
        } else {
            idle = 0;
        }
        n = nn;
    }
    // stopped: back to the global form -- cursor words, watched entries, entries, the item list
    if (v >= 0) g.lcur[v] = evcol ? GC_B_EVCOL : -np - 1;
    if (kind == 0 && g.b_watch > 0) B.watch[v] = acur;
    {
        const int pin = gc_wave_incl_scan(v >= 0 ? np : 0);
        const int pex = pin - (v >= 0 ? np : 0);
        const int ptot = __shfl(pin, GC_WAVE - 1, GC_WAVE);
        s.dst[lane] = B.pend + r0;
        s.np[lane] = off;
        gc_wave_sync();
        for (int b0 = 0; b0 < ptot; b0 += GC_WAVE) {
            const int e = b0 + lane;
            const int o = gc_owner(pex, e < ptot ? e : 0);
            const int x = e - __shfl(pex, o, GC_WAVE);
            if (e < ptot) s.dst[o][x] = pe[s.np[o] + x];
        }
    }
    const ull km = __ballot(v >= 0);
    if (v >= 0) l1[__popcll(km & gc_lanemask_lt())] = v | (kind << GC_BI_SHIFT);
    gc_wave_sync();
    return __popcll(km);
}

// pass `pass` of the round as one asynchronous launch: reads the three lists of slot
// pass % 3, spills to slot (pass + 1) % 3, uses the arrays of slot (pass + 2) % 3 as the
// waves' scratch and clears that slot's counts (as k_b_ev does)
// 6 waves per SIMD (80 VGPRs, 28 B of scratch per lane): R-MAT-26 -2.4 to -4.5% against 5, R-MAT-24 flat (r05/av)
#ifndef GC_B_WPE  // waves per SIMD the fold is compiled for (6: 80 VGPRs; a diagnostic build of the 7-8 per CU cliff raises it)
#define GC_B_WPE 6
#endif
__global__ void __launch_bounds__(GC_BLOCK) __attribute__((amdgpu_waves_per_eu(GC_B_WPE))) k_b_async(GDev g, BLists B, int* ev, int pass,
                                                                                       long long budget) {
    DevCtl* c = g.ctl;
    if (budget < 0) {  // residency probe (gcl_b_async_resident)
        gc_residency_probe(c);
        return;
    }
    if (c->halt) return;
    const int rs = pass % 3, ws = (pass + 1) % 3, zs = (pass + 2) % 3;
    __shared__ BAsyncLds s_w[GC_WAVES_PER_BLOCK];
    __shared__ int s_pe[GC_WAVES_PER_BLOCK][GC_B_RES_CAP];
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    const long long nA = (long long)*b_cnt(c, 0, rs), nH = (long long)*b_cnt(c, 1, rs), nE = (long long)*b_cnt(c, 2, rs);
    const long long T = nA + nH + nE;
    if (T > g.n) {  // never expected: report, touch nothing
        if (blockIdx.x == 0 && threadIdx.x == 0) __hip_atomic_store(&c->loop_err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    if (blockIdx.x == 0 && threadIdx.x < 3) *b_cnt(c, threadIdx.x, zs) = 0ull;
    const ull t0 = wall_clock64();
    budget += 2 * T;
    const long long W = (long long)gridDim.x * GC_WAVES_PER_BLOCK;
    const long long wid = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w;
    const long long a = T * wid / W, b = T * (wid + 1) / W;
    if (a >= b) return;
    int* l1 = B.l[0][zs] + a;  // light admissions and eviction times
    int* l2 = B.l[1][zs] + a;  // heavy admissions
    int n1 = 0, n2 = 0;
    for (long long i0 = a; i0 < b; i0 += GC_WAVE) {
        const long long i = i0 + lane;
        int v = -1, kind = -1;
        if (i < b) {
            if (i < nA) { v = B.l[0][rs][i]; kind = 0; }
            else if (i < nA + nH) { v = B.l[1][rs][i - nA]; kind = 1; }
            else { v = B.l[2][rs][i - nA - nH]; kind = 2; }
        }
        const ull m1 = __ballot(kind == 0 || kind == 2), m2 = __ballot(kind == 1);
        if (kind == 0 || kind == 2) l1[n1 + __popcll(m1 & gc_lanemask_lt())] = v | (kind << GC_BI_SHIFT);
        if (kind == 1) l2[n2 + __popcll(m2 & gc_lanemask_lt())] = v;
        n1 += __popcll(m1);
        n2 += __popcll(m2);
    }
    gc_wave_sync();
    bool stop = false;
    int idle = 0;
    int res_fail = GC_WAVE + 1;
    const bool use_res = g.b_resident != 0;
    ull lscan = 0, hscan = 0, npass = 0, htime = 0;
    const int h0 = n2, items0 = n1 + n2;
    while (n1 + n2 > 0) {
        const int before = n1 + n2;
        ++npass;
        n1 = b_async_chunk_pass(g, B, l1, n1, ev, s_w[w], &lscan, npass);
        if (n2) {
#ifdef GC_B_PROF
            const ull th = wall_clock64();
#endif
            n2 = b_async_heavy_pass(g, B, l2, n2, l1, &n1, ev, &hscan);
#ifdef GC_B_PROF
            htime += wall_clock64() - th;
#endif
        }
        if (n1 + n2 == 0) break;
        if ((stop = b_async_stop(c, t0, budget))) break;
        if (n1 + n2 == before) {
            if (++idle > 2) __builtin_amdgcn_s_sleep(2);
        } else {
            idle = 0;
        }
        if (use_res && n2 == 0 && n1 <= GC_WAVE && n1 < res_fail) {
            const int r = b_async_resident(g, B, l1, n1, ev, s_w[w], s_pe[w], c, t0, budget, &stop, &npass, &lscan);
            if (r >= 0) {
                n1 = r;
                break;  // settled, or stopped with the items written back
            }
            res_fail = n1;  // retried once fewer items are left
        }
    }
#ifdef GC_B_PROF
    if (lane == 0 && c->round < GC_B_PROF_ROUNDS) {
        ull* r = gc_bprof[c->round];
        const ull wall = wall_clock64() - t0;
        atomicMax(r + 0, wall);
        atomicMax(r + 1, htime);
        atomicMax(r + 2, npass);
        atomicAdd(r + 3, npass);
        atomicAdd(r + 4, (ull)h0);
        atomicMax(r + 5, (ull)items0);
        atomicMax(r + 6, lscan + hscan);
        atomicMax(r + 7, hscan);
        atomicMax(r + 8, (wall << 24) | (npass < (1u << 24) ? npass : (1u << 24) - 1));
        atomicMax(r + 9, (wall << 24) | ((htime >> 4) < (1u << 24) ? (htime >> 4) : (1u << 24) - 1));
        atomicAdd(r + 10, lscan + hscan);
        atomicAdd(r + 11, wall);
    }
#else
    (void)lscan; (void)hscan; (void)npass; (void)htime; (void)h0; (void)items0;
#endif
    if (!stop) return;
    // hand the unsettled items to the host's passes (slot ws), by kind
    for (int i0 = 0; i0 < n1; i0 += GC_WAVE) {
        const int it = i0 + lane < n1 ? l1[i0 + lane] : -1;
        const int kind = it >= 0 ? (it >> GC_BI_SHIFT) : -1;
        gc_wave_append(kind == 0, it & GC_BI_MASK, B.l[0][ws], b_cnt(c, 0, ws));
        gc_wave_append(kind == 2, it & GC_BI_MASK, B.l[2][ws], b_cnt(c, 2, ws));
    }
    for (int i0 = 0; i0 < n2; i0 += GC_WAVE) {
        const int v = i0 + lane < n2 ? l2[i0 + lane] : -1;
        gc_wave_append(v >= 0, v, B.l[1][ws], b_cnt(c, 1, ws));
    }
}

}  // namespace
int gcl_b_async_blocks_per_cu() { return gc_resident_blocks_per_cu((const void*)k_b_async, GC_BLOCK); }
static void launch_b_async_probe(const GDev& g, int grid, hipStream_t s) {
    BLists B{};
    GC_LAUNCH(k_b_async, dim3(grid), dim3(GC_BLOCK), 0, s, g, B, (int*)nullptr, 0, -1ll);
}
int gcl_b_async_resident(const GDev& g, hipStream_t s) {
    return gc_measure_resident((const void*)k_b_async, gc_graph_ctl_view{&g, s}, gcl_b_async_blocks_per_cu(),
                               launch_b_async_probe);
}
namespace {

struct RunB {
    gc_graph* g;
    GDev d;
    GLists L;
    hipStream_t s;
    // the round's wait: a one-workgroup kernel writes the control block into the pinned
    // snapshot slot (GC_SNAP_COPY=1: a copy-engine blit, as before), then an event wait
    const bool snap_copy = getenv("GC_SNAP_COPY") && atoi(getenv("GC_SNAP_COPY")) > 0;
    int sync() {
        GC_HIP(hipGetLastError());
        if (snap_copy || !g->hsnap_dev) {
            GC_HIP(hipMemcpyAsync(g->hctl, g->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, s));
            GC_HIP(hipStreamSynchronize(s));
            return GC_OK;
        }
        gcl_snap(g->ctl, g->hsnap_dev, s);
        GC_HIP(hipGetLastError());
        GC_HIP(hipEventRecord(g->evsnap[0], s));
        GC_HIP(hipEventSynchronize(g->evsnap[0]));
        memcpy(g->hctl, g->hsnap, sizeof(DevCtl));
        return GC_OK;
    }
    int zero(ull* p) {
        GC_HIP(hipMemsetAsync(p, 0, sizeof(ull), s));
        return GC_OK;
    }
};

}  // namespace

// The (deg, pos) rank partition (graph creation, gc_set_priority) already splits every low
// part by degree and counts the equal-degree entries (neq); variant A never looks inside a
// low part, so the layout serves both variants.
// GC_B_STALL_DUMP=prefix (diagnostics of the asynchronous fold's give-ups): the
// first time a round's fold is left unfinished by a k_b_async launch that stopped at its budget,
// write the state the host's passes start from -- the unsettled items (the three lists of the
// spill slot), k8, cand, the eviction times, cursors, watched entries and pending entries -- as
// raw arrays <prefix>.<name>.bin, for tools/b_stall_analyze.py
static int b_stall_dump(gc_graph* g, const BLists& B, const int* ev, const DevCtl& h, long long passes, long long round) {
    static bool done = false;
    const char* pre = getenv("GC_B_STALL_DUMP");
    if (!pre || done || h.async_aborts == 0) return GC_OK;
    done = true;
    const int ws = (int)(passes % 3);
    auto dump = [&](const char* name, const void* dev, size_t bytes) -> int {
        std::vector<char> buf(bytes);
        if (bytes) GC_READ(g->stream, buf.data(), (const char*)dev, bytes);
        std::string path = std::string(pre) + "." + name + ".bin";
        if (FILE* f = fopen(path.c_str(), "wb")) {
            fwrite(buf.data(), 1, bytes, f);
            fclose(f);
        }
        return GC_OK;
    };
    int rc;
    for (int k = 0; k < 3; ++k) {
        const char* nm[3] = {"adm", "heavy", "evict"};
        if ((rc = dump(nm[k], B.l[k][ws], sizeof(int) * (size_t)h.bcnt[3 * k + ws]))) return rc;
    }
    if ((rc = dump("k8", g->k8, (size_t)g->n)) || (rc = dump("cand", g->cand, sizeof(int) * (size_t)g->n)) ||
        (rc = dump("ev", ev, sizeof(int) * (size_t)g->n)) || (rc = dump("lcur", g->lcur, sizeof(int) * (size_t)g->n)) ||
        (rc = dump("watch", B.watch, sizeof(int) * (size_t)g->n)) ||
        (rc = dump("nhe", B.nhe, sizeof(int) * (size_t)g->n)) || (rc = dump("neq", g->neq, sizeof(int) * (size_t)g->n)))
        return rc;
    {  // the listed items' pending entries only: [v, count, entries...] per item (the whole array is nnz ints)
        std::vector<long long> rp((size_t)g->n + 1);
        std::vector<int> lcur((size_t)g->n), pend((size_t)g->nnz);
        GC_READ(g->stream, rp.data(), g->rp, rp.size());
        GC_READ(g->stream, lcur.data(), g->lcur, lcur.size());
        if (g->nnz) GC_READ(g->stream, pend.data(), B.pend, pend.size());
        std::vector<int> outv;
        for (int k = 0; k < 3; ++k) {
            std::vector<int> items((size_t)h.bcnt[3 * k + ws]);
            if (!items.empty()) GC_READ(g->stream, items.data(), B.l[k][ws], items.size());
            for (int v : items) {
                const int lc = lcur[(size_t)v];
                const int cnt = lc < 0 ? -lc - 1 : 0;
                outv.push_back(v);
                outv.push_back(cnt);
                for (int i = 0; i < cnt; ++i) outv.push_back(pend[(size_t)rp[(size_t)v] + i]);
            }
        }
        std::string path = std::string(pre) + ".pendrows.bin";
        if (FILE* f = fopen(path.c_str(), "wb")) {
            fwrite(outv.data(), sizeof(int), outv.size(), f);
            fclose(f);
        }
    }
    std::string path = std::string(pre) + ".info.txt";
    if (FILE* f = fopen(path.c_str(), "w")) {
        fprintf(f, "round %lld passes %lld aborts %llu n %lld nnz %lld adm %llu heavy %llu evict %llu\n", round, passes,
                (unsigned long long)h.async_aborts, g->n, g->nnz, (unsigned long long)h.bcnt[ws],
                (unsigned long long)h.bcnt[3 + ws], (unsigned long long)h.bcnt[6 + ws]);
        fclose(f);
    }
    return GC_OK;
}

static int ensure_bpart(gc_graph* g) {
    if (g->part_prio != GC_PRIORITY_REF || !g->bpart || !g->neq || !g->nhe) {
        gc_set_error("variant B needs the (deg, pos) row partition");
        return GC_EINVAL;
    }
    return GC_OK;
}

int gc_color_variant_b(gc_graph* g, const gc_options* opt, int32_t* colors_out, int32_t* cround_out, gc_stats* st) {
    RunB R{g, gc_view(g), gc_lists(g), g->stream};
    int rc;
    // hubs keep their forbidden colours as pushed bitmaps (every uncoloured vertex proposes
    // every round: without them k_propose_block re-reads every hub row each round)
    if ((rc = gc_hubs_prepare(g, R.d))) return rc;
    R.d.hub_w = 0;  // bitmaps only: the fold has no hub JP
    R.d.tail_hmax = GC_TAIL_HMAX;
    // the asynchronous fold's resident form (b_async_resident); GC_B_RESIDENT=0 off
    R.d.b_resident = getenv("GC_B_RESIDENT") ? atoi(getenv("GC_B_RESIDENT")) : 1;
    // watched entries (b_async_chunk_pass): a full admission rescan every GC_B_WATCH-th pass at most
    // otherwise; 0 off
    R.d.b_watch = getenv("GC_B_WATCH") ? atoi(getenv("GC_B_WATCH")) : 4;
    R.d.b_awin = getenv("GC_B_AWIN") ? atoi(getenv("GC_B_AWIN")) : 8;  // the window's entries
    if (R.d.b_awin < 1) R.d.b_awin = 1;
    R.d.b_refskip = getenv("GC_B_REFSKIP") ? atoi(getenv("GC_B_REFSKIP")) : 1;
    const hipStream_t s = R.s;
    const GDev& d = R.d;
    const GLists& L = R.L;
    // fold pass grids (env GC_GRID_BE / GC_GRID_BA: eviction / admission passes).  Heavy
    // admissions take a workgroup each: with vertices that can be heavy, 2048 workgroups
    // (R-MAT-24 891 -> 824 ms; 4096: 928, 512: 1134); C2 keeps 1024 (4096: 18.4 -> 22.0 ms)
    const int grid_ev = getenv("GC_GRID_BE") && atoi(getenv("GC_GRID_BE")) > 0 ? atoi(getenv("GC_GRID_BE")) : GC_ROUND_GRID;
    const int grid_adm = getenv("GC_GRID_BA") && atoi(getenv("GC_GRID_BA")) > 0 ? atoi(getenv("GC_GRID_BA"))
                         : (g->maxdeg > GC_B_HEAVY ? 2 * GC_ROUND_GRID : GC_ROUND_GRID);
    // The round's fold as one asynchronous launch (k_b_async) on a resident grid (CUs x 4
    // workgroups, GC_B_ASYNC_BPC, capped by the occupancy: R-MAT-24 420 ms at 2, 363 at 4, 557 at
    // 1, profiles/r04/l) after GC_B_ASYNC_K (default 0) full-grid passes; budget per launch
    // GC_ASYNC_BUDGET_US (20 ms) plus 2 cycles per work item.  On by default for graphs with
    // hubs (round 4: R-MAT-24 658 -> 455 ms with K = 0, 497 with K = 1, 473 with K = 2;
    // uniform 10M/16, no hub, 20.0 -> 21.4 ms: off there, as variant A's asynchronous JP;
    // profiles/r04/k).  GC_B_ASYNC=0 off, =1 on for every graph.
    int b_async_grid = 0;
    long long b_async_budget = 0;
    const long long b_async_k = getenv("GC_B_ASYNC_K") ? std::max(0ll, atoll(getenv("GC_B_ASYNC_K"))) : 0;
    const int b_async_env = getenv("GC_B_ASYNC") ? atoi(getenv("GC_B_ASYNC")) : -1;
    const bool b_async_on = b_async_env > 0 || (b_async_env < 0 && d.hbits_w > 0);
    if (b_async_on && g->n < (1ll << GC_BI_SHIFT)) {  // items: 29-bit vertices
        int cus = 0, rate_khz = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, g->device) == hipSuccess &&
            hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, g->device) == hipSuccess && cus > 0 &&
            rate_khz > 0) {
            const int bpc = getenv("GC_B_ASYNC_BPC") && atoi(getenv("GC_B_ASYNC_BPC")) > 0 ? atoi(getenv("GC_B_ASYNC_BPC")) : 6;
            // every workgroup resident (gc_resident_blocks_per_cu): the static slices all progress
            b_async_grid = std::min(bpc, std::max(1, gcl_b_async_resident(d, s))) * cus;
            const long long us = getenv("GC_ASYNC_BUDGET_US") ? atoll(getenv("GC_ASYNC_BUDGET_US")) : 20000;
            b_async_budget = std::max(0ll, us) * (long long)rate_khz / 1000;
        }
    }
    DevCtl& h = *g->hctl;
    memset(&h, 0, sizeof(DevCtl));
    h.kbound = opt->num_colors;
    h.rcap = g->rcap;
    h.maxmex = -1;
    h.maxcolor = -1;
    h.fail_round = -1;
    h.want_cround = cround_out != nullptr;
    GC_HIP(hipMemcpyAsync(g->ctl, &h, sizeof(DevCtl), hipMemcpyHostToDevice, s));
    GC_HIP(hipMemsetAsync(g->bstat, 0, sizeof(ull) * GC_STAT_SLOTS * 16, s));
    GC_HIP(hipEventRecord(g->ev0, s));
    // init + seed (coloring_optimized.py:70-80 == coloring.py:12-35)
    // per-class launch timing (gc_options.kernel_timing), as the one-GPU engine: the fold
    // (k_b_init and its passes or k_b_async) is the resolution class
    KTimer kt{g, (unsigned)opt->kernel_timing, st};
    kt.begin(GC_K_INIT);
    gcl_init(d, g->seeds[0], gc_grid_for_waves(g->n), s);
    gcl_seed_prep(d, g->seeds[0], g->seeds[1], s);
    gcl_commit(d, L, GC_CM_INIT, 0, s);
    // every vertex counts as claimed: the re-sort then lists exactly the uncoloured ones
    GC_HIP(hipMemsetAsync(g->inF, 0xFF, sizeof(unsigned) * (size_t)((g->n + 63) / 32 + 2), s));
    int* ev = g->parent;  // E1 scratch, unused by variant B
    if ((rc = ensure_bpart(g))) return rc;
    // work lists (variant A's undecided, seed and E1 lists are free during variant B)
    BLists B;
    int* const wl[9] = {g->undL[0], g->undL[1], g->undL[2], g->seeds[0], g->seeds[1], g->bigw,
                        g->undH[0], g->undH[1], g->undH[2]};
    for (int k = 0; k < 9; ++k) B.l[k / 3][k % 3] = wl[k];
    if (!g->bpend && g->nnz > 0) GC_HIP(gc_dmalloc((void**)&g->bpend, sizeof(int) * (size_t)g->nnz));
    B.pend = g->bpend;
    if (!g->bwatch && g->n > 0) {
        GC_HIP(gc_dmalloc((void**)&g->bwatch, sizeof(int) * (size_t)g->n));
        GC_HIP(hipMemsetAsync(g->bwatch, 0xFF, sizeof(int) * (size_t)g->n, s));  // -1: none
    }
    B.watch = g->bwatch;
    B.nhe = g->nhe;
    std::vector<RoundRec> recs;
    int status = GC_OK;
    long long sweeps_total = 0, fail_round = -1, fail_count = 0;
    const long long max_rounds = 4ll * g->n + 16;
    // One host wait per round in the common case: the round's re-sort, proposals and its
    // first batch of fold passes are enqueued together (as many passes as the previous
    // round needed); the previous round's winner count comes back in the same snapshot
    // (k_b_reset keeps it).  A round that ends the colouring (no uncoloured vertex) or
    // fails (bounded attempt) has only run fold passes, which change no colour.
    long long prev_passes = 2, prevU = 0, prev_maxmex = -1;
    // Pipelined rounds (GC_B_PIPE, default on): round r + 1 is enqueued before the host reads
    // round r's snapshot, and round r's commit makes the round's decisions itself
    // (k_b_commit's check_ws): the device never idles on the host's round trip (~25 ms of
    // R-MAT-24's colouring, one per round).  A round the commit halts -- done, failed, or a fold
    // the enqueued passes did not finish -- leaves the next round a no-op (k_b_reset), which the
    // host discards; an unfinished fold is finished by host passes as below and the pipeline
    // restarts after its commit.
    const bool pipe = !(getenv("GC_B_PIPE") && atoi(getenv("GC_B_PIPE")) == 0) && g->hsnap_dev != nullptr;
    long long passes_of[2] = {0, 0};
    auto enqueue_passes_into = [&](long long& passes, long long k) {
        for (long long j = 0; j < k; ++j, ++passes) {
            const int pi = (int)(passes % 3);
            GC_LAUNCH(k_b_ev, dim3(grid_ev), dim3(GC_BLOCK), 0, s, d, B, ev, pi);
            GC_LAUNCH(k_b_adm, dim3(grid_adm), dim3(GC_BLOCK), 0, s, d, B, (const int*)ev, pi);
        }
    };
    auto enqueue_round = [&](long long rr) -> int {
        kt.begin(GC_K_OTHER);
        GC_LAUNCH(k_b_reset, dim3(1), dim3(64), 0, s, d, rr);
        gcl_fsort(d, L, g->fsum, s);
        gcl_pack_c4(d, s);
        kt.begin(GC_K_PROPOSE);
        gcl_propose(d, L, s);
        gcl_propose_block(d, L, s);
        if (h.kbound == 0) {
            GC_HIP(hipMemsetAsync(&g->ctl->failcnt, 0, sizeof(ull), s));
            GC_LAUNCH(k_b_fail0, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, d, L);
        }
        kt.begin(GC_K_RESOLVE);
        GC_LAUNCH(k_b_init, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, d, L, B, ev, (const int*)g->neq);
        long long passes = 0;
        if (b_async_grid > 0) {
            enqueue_passes_into(passes, b_async_k);
            if (b_async_k > 0) GC_HIP(hipMemsetAsync(&g->ctl->async_abort[0], 0, sizeof(int), s));
            GC_LAUNCH(k_b_async, dim3(b_async_grid), dim3(GC_BLOCK), 0, s, d, B, ev, (int)(passes % 3), b_async_budget);
            ++passes;
        } else {
            enqueue_passes_into(passes, std::max(2ll, std::min(prev_passes, 24ll)));
        }
        kt.begin(GC_K_COMMIT);
        GC_LAUNCH(k_b_commit, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, d, L, (const int*)ev, g->ulist, (int)(passes % 3));
        if (d.hbits_w) gcl_hub_push_big(d, g->ulist, &g->ctl->bigw_cnt, s);
        kt.close();
        gcl_snap(g->ctl, g->hsnap_dev + (rr & 1), s);
        GC_HIP(hipGetLastError());
        GC_HIP(hipEventRecord(g->evsnap[rr & 1], s));
        passes_of[rr & 1] = passes;
        return GC_OK;
    };
    if (pipe) {
        if ((rc = enqueue_round(0))) return rc;
        long long next = 1;
        for (long long cur = 0;;) {
            if (next > max_rounds) { gc_set_error("round limit exceeded"); return GC_EROUNDS; }
            if ((rc = enqueue_round(next))) return rc;  // one round ahead: two in flight, two slots
            ++next;
            GC_HIP(hipEventSynchronize(g->evsnap[cur & 1]));
            DevCtl sn;
            memcpy(&sn, &g->hsnap[cur & 1], sizeof(DevCtl));
            if (sn.loop_err == GC_LERR_LIST) { gc_set_error("variant B: a work-list append passed the list's capacity"); return GC_EHIP; }
            if (sn.loop_err == 2) { gc_set_error("k_b_async: work list count out of range"); return GC_EHIP; }
            const long long U = (long long)sn.fcnt[0];
            const long long np = passes_of[cur & 1];
            if (sn.halt == GC_RUN) {
                recs.push_back(RoundRec{U, U, (long long)sn.maxmex, (long long)sn.accepted, 0, np});
                sweeps_total += np;
                prev_passes = np;
                ++cur;
                continue;
            }
            if (sn.halt == GC_H_DONE) {  // coloring_optimized.py: no uncoloured vertex left
                recs.push_back(RoundRec{0, 0, -1, 0, 0, 0});
                break;
            }
            if (sn.halt == GC_H_FAILED) {  // state at the round start is returned
                recs.push_back(RoundRec{U, U, (long long)sn.maxmex, 0, 0, 0});
                status = GC_FAILED;
                fail_round = cur;
                fail_count = (long long)sn.failcnt;
                break;
            }
            if (sn.halt != GC_H_SWEEPS) { gc_set_error("variant B: unexpected halt %d", sn.halt); return GC_EHIP; }
            // round cur's fold is unfinished (round cur + 1 ran as a no-op): its passes, its commit
            if ((rc = R.sync())) return rc;
            if ((rc = b_stall_dump(g, B, ev, h, np, cur))) return rc;
            GC_HIP(hipMemsetAsync(&g->ctl->halt, 0, sizeof(int), s));
            long long passes = np;
            for (long long batch = 4;; batch = std::min(batch * 2, 16ll)) {
                const int ws = (int)(passes % 3);
                if (h.bcnt[ws] + h.bcnt[3 + ws] + h.bcnt[6 + ws] == 0) break;
                if (passes > 2 * g->n + 64) { gc_set_error("variant B passes do not converge"); return GC_EROUNDS; }
                kt.begin(GC_K_RESOLVE);
                enqueue_passes_into(passes, batch);
                kt.close();
                if ((rc = R.sync())) return rc;
            }
            kt.begin(GC_K_COMMIT);
            GC_LAUNCH(k_b_commit, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, d, L, (const int*)ev, g->ulist, -1);
            if (d.hbits_w) gcl_hub_push_big(d, g->ulist, &g->ctl->bigw_cnt, s);
            kt.close();
            if ((rc = R.sync())) return rc;
            recs.push_back(RoundRec{U, U, (long long)sn.maxmex, (long long)h.accepted, 0, passes});
            sweeps_total += passes;
            prev_passes = passes;
            ++cur;
            next = cur;  // the no-op round again
            if ((rc = enqueue_round(next))) return rc;
            ++next;
        }
    }
    for (long long r = 0; !pipe; ++r) {
        if (r > max_rounds) { gc_set_error("round limit exceeded"); return GC_EROUNDS; }
        kt.begin(GC_K_OTHER);
        GC_LAUNCH(k_b_reset, dim3(1), dim3(64), 0, s, d, r);
        gcl_fsort(d, L, g->fsum, s);
        gcl_pack_c4(d, s);
        kt.begin(GC_K_PROPOSE);
        gcl_propose(d, L, s);
        gcl_propose_block(d, L, s);
        if (h.kbound == 0) {
            if ((rc = R.zero(&g->ctl->failcnt))) return rc;
            GC_LAUNCH(k_b_fail0, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, d, L);
        }
        // the fold's passes over the work lists until no vertex is undecided and every
        // admitted vertex's eviction time is final
        kt.begin(GC_K_RESOLVE);
        GC_LAUNCH(k_b_init, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, d, L, B, ev, (const int*)g->neq);
        long long passes = 0;
        auto enqueue_passes = [&](long long k) {
            for (long long j = 0; j < k; ++j, ++passes) {
                const int pi = (int)(passes % 3);  // slot arithmetic only needs the pass mod 3
                GC_LAUNCH(k_b_ev, dim3(grid_ev), dim3(GC_BLOCK), 0, s, d, B, ev, pi);
                GC_LAUNCH(k_b_adm, dim3(grid_adm), dim3(GC_BLOCK), 0, s, d, B, (const int*)ev, pi);
            }
        };
        // an open timing run never spans a host wait (the resolve class took every
        // round's synchronisation and host decision time)
        auto synced = [&]() {
            kt.close();
            return R.sync();
        };
        if (b_async_grid > 0) {  // the first passes on the full grid, then the rest as one asynchronous launch
            enqueue_passes(b_async_k);
            if (b_async_k > 0) GC_HIP(hipMemsetAsync(&g->ctl->async_abort[0], 0, sizeof(int), s));
            GC_LAUNCH(k_b_async, dim3(b_async_grid), dim3(GC_BLOCK), 0, s, d, B, ev, (int)(passes % 3),
                               b_async_budget);
            ++passes;
        } else {
            enqueue_passes(std::max(2ll, std::min(prev_passes, 24ll)));
        }
        if ((rc = synced())) return rc;
        if (r > 0) {
            recs.push_back(RoundRec{prevU, prevU, prev_maxmex, (long long)h.dcnt, 0, prev_passes});
            sweeps_total += prev_passes;
        }
        if (h.loop_err == GC_LERR_LIST) { gc_set_error("variant B: a work-list append passed the list's capacity"); return GC_EHIP; }
        if (h.loop_err == 2) { gc_set_error("k_b_async: work list count out of range"); return GC_EHIP; }
        const long long U = (long long)h.fcnt[0];
        if (U == 0) {  // coloring_optimized.py: no uncoloured vertex left
            recs.push_back(RoundRec{0, 0, -1, 0, 0, 0});
            break;
        }
        const long long maxmex = h.maxmex;
        if (h.kbound >= 0 && h.failcnt > 0) {  // state at the round start is returned
            recs.push_back(RoundRec{U, U, maxmex, 0, 0, 0});
            status = GC_FAILED;
            fail_round = r;
            fail_count = (long long)h.failcnt;
            break;
        }
        for (long long batch = 4;; batch = std::min(batch * 2, 16ll)) {
            const int ws = (int)(passes % 3);  // written by the last pass
            if (h.bcnt[ws] + h.bcnt[3 + ws] + h.bcnt[6 + ws] == 0) break;
            if (passes > 2 * g->n + 64) { gc_set_error("variant B passes do not converge"); return GC_EROUNDS; }
            kt.begin(GC_K_RESOLVE);
            enqueue_passes(batch);
            if ((rc = synced())) return rc;
        }
        kt.begin(GC_K_COMMIT);
        GC_LAUNCH(k_b_commit, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, d, L, (const int*)ev, g->ulist, -1);
        if (d.hbits_w) gcl_hub_push_big(d, g->ulist, &g->ctl->bigw_cnt, s);
        prev_passes = passes;
        prevU = U;
        prev_maxmex = maxmex;
    }
    kt.begin(GC_K_OTHER);
    gcl_finalize(d, gc_grid_for_waves(g->n, 8192), s);
    gcl_stat_reduce(d, s);
    kt.close();
    GC_HIP(hipEventRecord(g->ev1, s));
    if (colors_out) GC_HIP(hipMemcpyAsync(colors_out, g->color, sizeof(int) * g->n, hipMemcpyDeviceToHost, s));
    if (cround_out) GC_HIP(hipMemcpyAsync(cround_out, g->cround, sizeof(int) * g->n, hipMemcpyDeviceToHost, s));
    if ((rc = R.sync())) return rc;
#ifdef GC_B_PROF
    if (const char* pp = getenv("GC_B_PROF_OUT")) {  // append this colouring's per-round records
        static ull hb[GC_B_PROF_ROUNDS][GC_B_PROF_K];
        GC_HIP(hipMemcpyFromSymbol(hb, HIP_SYMBOL(gc_bprof), sizeof(hb)));
        if (FILE* f = fopen(pp, "a")) {
            fprintf(f, "# colouring: %zu rounds; per round: U wall_us heavy_us max_passes sum_passes heavy_items max_items "
                    "max_scanned max_heavy_scanned slowest_passes slowest_heavy_us sum_scanned sum_wall_us\n", recs.size());
            for (size_t i = 0; i < recs.size() && i < GC_B_PROF_ROUNDS; ++i) {
                const ull* r = hb[i];
                fprintf(f, "%zu %lld %.1f %.1f %llu %llu %llu %llu %llu %llu %llu %.1f %llu %.1f\n", i, recs[i].U,
                        r[0] / 100.0, r[1] / 100.0, r[2], r[3], r[4], r[5], r[6], r[7], r[8] & 0xFFFFFF,
                        (r[9] & 0xFFFFFF) * 16 / 100.0, r[10], r[11] / 100.0);
            }
            fclose(f);
        }
        static ull z[GC_B_PROF_ROUNDS][GC_B_PROF_K];
        GC_HIP(hipMemcpyToSymbol(HIP_SYMBOL(gc_bprof), z, sizeof(z)));
    }
#endif
    if (st) {
        kt.collect();
        float ms = 0.f;
        GC_HIP(hipEventElapsedTime(&ms, g->ev0, g->ev1));
        st->device_ms = ms;
        st->rounds = (long long)recs.size();
        st->max_color = h.maxcolor;
        st->jp_sweeps = sweeps_total;
        st->async_aborts = (int64_t)h.async_aborts;
        st->hubs = R.d.hbits_w ? (int64_t)g->nhub : 0;
        st->fail_round = fail_round;
        st->fail_count = fail_count;
        for (long long i = 0; i < (long long)recs.size() && i < st->round_cap; ++i) {
            const RoundRec& rr = recs[(size_t)i];
            if (st->round_U) st->round_U[i] = rr.U;
            if (st->round_F) st->round_F[i] = rr.F;
            if (st->round_maxmex) st->round_maxmex[i] = rr.maxmex;
            if (st->round_accepted) st->round_accepted[i] = rr.accepted;
            if (st->round_seeds) st->round_seeds[i] = rr.seeds;
        }
        // SURVEY.md §8d algorithmic bytes: propose and resolve both visit every proposer
        st->k_bytes[GC_K_PROPOSE] = 24.0 * (double)h.nvert[GC_K_PROPOSE] + 8.0 * (double)h.sumdeg[GC_K_PROPOSE];
        st->k_bytes[GC_K_RESOLVE] = 24.0 * (double)h.nvert[GC_K_PROPOSE] + 12.0 * (double)h.sumdeg[GC_K_PROPOSE];
        st->k_bytes[GC_K_COMMIT] = 16.0 * (double)h.nvert[GC_K_COMMIT] + 8.0 * (double)h.sumdeg[GC_K_COMMIT];
    }
    return status;
}
