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
    c->halt = GC_RUN;
    c->round = round;
    c->cur = 0;
    c->fcnt[0] = 0;
    c->fcnt[1] = 0;
    c->heavy_cnt = 0;
    c->wide_cnt = 0;
    c->failcnt = 0;
    c->maxmex = -1;
    c->accepted = 0;
    c->fsort_all = 1;
    for (int k = 0; k < 3; ++k) c->und_cnt[k] = 0;
}

// bounded attempt with k = 0: only proposers WITH a coloured neighbour fail
// (coloring_optimized.py:159-164); k_propose counted every proposer.
__global__ void __launch_bounds__(GC_BLOCK) k_b_fail0(GDev g, GLists L) {
    DevCtl* c = g.ctl;
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

// ev pass over the admitted vertices whose eviction time is not final
__global__ void __launch_bounds__(GC_BLOCK) k_b_ev(GDev g, GLists L, int* ev) {
    DevCtl* c = g.ctl;
    __shared__ long long s_start[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_min[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_v[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_d[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ unsigned s_c6[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_cv[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ ull scratch[2 * GC_WAVES_PER_BLOCK];
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    const int* __restrict__ list = L.F[c->cur];
    const long long cnt = (long long)c->fcnt[c->cur];
    const unsigned char* __restrict__ k8 = g.k8;
    ull pend = 0;
    const int vpw = gc_vpw(cnt, (long long)gridDim.x * GC_WAVES_PER_BLOCK);
    const long long nch = gc_nchunks(cnt, vpw);
    for (long long ch = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w; ch < nch;
         ch += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
        const long long idx = ch * vpw + lane;
        const int v = (lane < vpw && idx < cnt) ? list[idx] : -1;
        const unsigned kv = v >= 0 ? (unsigned)k8[v] : 0u;
        bool act = false;
        if (v >= 0 && gc_k8_state(kv) == GC_JP_IN) {
            const int e = ev[v];
            act = e < 0 || (e != GC_B_INF && gc_k8_state(k8[e]) != GC_JP_IN);
        }
        const int d = act ? g.deg[v] : 0;
        s_start[w][lane] = act ? g.rp[v] : 0;
        s_min[w][lane] = GC_B_INF;
        s_v[w][lane] = v;
        s_d[w][lane] = d;
        s_c6[w][lane] = act ? gc_k8_cand(kv) : 0x100u;
        s_cv[w][lane] = act ? b_cand(g, v, kv) : -1;
        const int incl = gc_wave_incl_scan(d);
        const int excl = incl - d;
        const int total = __shfl(incl, GC_WAVE - 1, GC_WAVE);
        gc_wave_sync();
        gc_chunk_edges(
            g.col, s_start[w], excl, total, [&](int u) { return (unsigned)k8[u]; },
            [&](int o, int u, unsigned ku) {
                if (u <= s_v[w][o] || gc_k8_state(ku) == GC_JP_OUT) return;
                if (!b_same(g, u, ku, s_c6[w][o], s_cv[w][o])) return;
                if (g.deg[u] > s_d[w][o]) atomicMin(&s_min[w][o], u);
            });
        gc_wave_sync();
        if (act) {
            const int e = s_min[w][lane];
            ev[v] = e;
            if (e != GC_B_INF && gc_k8_state(k8[e]) != GC_JP_IN) pend++;
        }
    }
    __syncthreads();
    gc_block_add(&c->und_cnt[1], pend, scratch);
}

// admission pass over the undecided vertices
__global__ void __launch_bounds__(GC_BLOCK) k_b_adm(GDev g, GLists L, const int* ev) {
    DevCtl* c = g.ctl;
    __shared__ long long s_start[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ unsigned s_flag[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_v[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_d[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ unsigned s_c6[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_cv[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ ull scratch[2 * GC_WAVES_PER_BLOCK];
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    const int* __restrict__ list = L.F[c->cur];
    const long long cnt = (long long)c->fcnt[c->cur];
    const unsigned char* __restrict__ k8 = g.k8;
    ull und = 0;
    const int vpw = gc_vpw(cnt, (long long)gridDim.x * GC_WAVES_PER_BLOCK);
    const long long nch = gc_nchunks(cnt, vpw);
    for (long long ch = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w; ch < nch;
         ch += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
        const long long idx = ch * vpw + lane;
        const int v = (lane < vpw && idx < cnt) ? list[idx] : -1;
        const unsigned kv = v >= 0 ? (unsigned)k8[v] : 0u;
        const bool act = v >= 0 && gc_k8_state(kv) == GC_JP_UND;
        const int d = act ? g.deg[v] : 0;
        s_start[w][lane] = act ? g.rp[v] : 0;
        s_flag[w][lane] = 0;
        s_v[w][lane] = v;
        s_d[w][lane] = d;
        s_c6[w][lane] = act ? gc_k8_cand(kv) : 0x100u;
        s_cv[w][lane] = act ? b_cand(g, v, kv) : -1;
        const int incl = gc_wave_incl_scan(d);
        const int excl = incl - d;
        const int total = __shfl(incl, GC_WAVE - 1, GC_WAVE);
        gc_wave_sync();
        gc_chunk_edges(
            g.col, s_start[w], excl, total, [&](int u) { return (unsigned)k8[u]; },
            [&](int o, int u, unsigned ku) {
                const int vo = s_v[w][o];
                if (u >= vo) return;  // later arrivals (and self-loops) never count
                const unsigned st = gc_k8_state(ku);
                if (st == GC_JP_OUT || !b_same(g, u, ku, s_c6[w][o], s_cv[w][o])) return;
                if (g.deg[u] < s_d[w][o]) return;
                unsigned f = 2u;  // undecided, or admitted with an eviction time not yet known
                if (st == GC_JP_IN) {
                    const int e = ev[u];
                    if (e > vo) f = 1u;                                   // still admitted at v's arrival
                    else if (e >= 0 && gc_k8_state(k8[e]) == GC_JP_IN) f = 0u;  // evicted before v
                }
                if (f) atomicOr(&s_flag[w][o], f);
            });
        gc_wave_sync();
        if (act) {
            const unsigned f = s_flag[w][lane];
            if (f & 1u) g.k8[v] = (unsigned char)((kv & ~3u) | GC_JP_OUT);
            else if (f & 2u) und++;
            else g.k8[v] = (unsigned char)((kv & ~3u) | GC_JP_IN);
        }
    }
    __syncthreads();
    gc_block_add(&c->und_cnt[0], und, scratch);
}

// winners: admitted and never evicted, coloured (coloring_optimized.py:129-140)
__global__ void __launch_bounds__(GC_BLOCK) k_b_commit(GDev g, GLists L, const int* ev) {
    DevCtl* c = g.ctl;
    __shared__ ull scratch[2 * GC_WAVES_PER_BLOCK];
    const long long cnt = (long long)c->fcnt[c->cur];
    const int* list = L.F[c->cur];
    const int round = (int)(c->round + 1);
    const bool want_cround = c->want_cround != 0;
    long long lmaxc = -1;
    ull lacc = 0, lsum = 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += (long long)gridDim.x * blockDim.x) {
        const int v = list[i];
        const unsigned kv = g.k8[v];
        if (gc_k8_state(kv) != GC_JP_IN || ev[v] != GC_B_INF) continue;
        const int cc = b_cand(g, v, kv);
        gc_commit_colour(g, v, cc);
        if (want_cround) g.cround[v] = round;
        lmaxc = cc > lmaxc ? cc : lmaxc;
        lacc++;
        lsum += (ull)g.deg[v];
    }
    __syncthreads();
    gc_block_max(&c->maxcolor, lmaxc, (long long*)scratch);
    gc_block_add(&c->accepted, lacc, scratch);
    gc_stat_add(g, GC_K_COMMIT, lsum, lacc, scratch);
}

struct RunB {
    gc_graph* g;
    GDev d;
    GLists L;
    hipStream_t s;
    int sync() {
        GC_HIP(hipGetLastError());
        GC_HIP(hipMemcpyAsync(g->hctl, g->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, s));
        GC_HIP(hipStreamSynchronize(s));
        return GC_OK;
    }
    int zero(ull* p) {
        GC_HIP(hipMemsetAsync(p, 0, sizeof(ull), s));
        return GC_OK;
    }
};

}  // namespace

int gc_color_variant_b(gc_graph* g, const gc_options* opt, int32_t* colors_out, int32_t* cround_out, gc_stats* st) {
    RunB R{g, gc_view(g), gc_lists(g), g->stream};
    const hipStream_t s = R.s;
    const GDev& d = R.d;
    const GLists& L = R.L;
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
    gcl_init(d, g->seeds[0], gc_grid_for_waves(g->n), s);
    gcl_seed_prep(d, g->seeds[0], g->seeds[1], s);
    gcl_commit(d, L, GC_CM_INIT, 0, s);
    // every vertex counts as claimed: the re-sort then lists exactly the uncoloured ones
    GC_HIP(hipMemsetAsync(g->inF, 0xFF, sizeof(unsigned) * (size_t)((g->n + 63) / 32 + 2), s));
    int* ev = g->parent;  // E1 scratch, unused by variant B
    std::vector<RoundRec> recs;
    int status = GC_OK, rc;
    long long sweeps_total = 0, fail_round = -1, fail_count = 0;
    const long long max_rounds = 4ll * g->n + 16;
    for (long long r = 0;; ++r) {
        if (r > max_rounds) { gc_set_error("round limit exceeded"); return GC_EROUNDS; }
        hipLaunchKernelGGL(k_b_reset, dim3(1), dim3(64), 0, s, d, r);
        gcl_fsort(d, L, g->fsum, s);
        if ((rc = R.sync())) return rc;
        const long long U = (long long)h.fcnt[0];
        if (U == 0) {  // coloring_optimized.py: no uncoloured vertex left
            recs.push_back(RoundRec{0, 0, -1, 0, 0, 0});
            break;
        }
        gcl_pack_c4(d, s);
        gcl_propose(d, L, s);
        gcl_propose_block(d, L, s);
        if (h.kbound == 0) {
            if ((rc = R.zero(&g->ctl->failcnt))) return rc;
            hipLaunchKernelGGL(k_b_fail0, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, d, L);
        }
        if ((rc = R.sync())) return rc;
        const long long maxmex = h.maxmex;
        if (h.kbound >= 0 && h.failcnt > 0) {  // state at the round start is returned
            recs.push_back(RoundRec{U, U, maxmex, 0, 0, 0});
            status = GC_FAILED;
            fail_round = r;
            fail_count = (long long)h.failcnt;
            break;
        }
        GC_HIP(hipMemsetAsync(ev, 0xFF, sizeof(int) * (size_t)g->n, s));
        long long passes = 0;
        for (int batch = 2;; batch = std::min(batch * 2, 16)) {
            for (int j = 0; j < batch; ++j) {
                if ((rc = R.zero(&g->ctl->und_cnt[0])) || (rc = R.zero(&g->ctl->und_cnt[1]))) return rc;
                hipLaunchKernelGGL(k_b_ev, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, d, L, ev);
                hipLaunchKernelGGL(k_b_adm, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, d, L, (const int*)ev);
            }
            passes += batch;
            if ((rc = R.sync())) return rc;
            if (h.und_cnt[0] == 0) break;
            if (passes > g->n + 64) { gc_set_error("variant B passes do not converge"); return GC_EROUNDS; }
        }
        // every admission is decided: one more ev pass makes every eviction time final
        if ((rc = R.zero(&g->ctl->und_cnt[1]))) return rc;
        hipLaunchKernelGGL(k_b_ev, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, d, L, ev);
        hipLaunchKernelGGL(k_b_commit, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, d, L, (const int*)ev);
        if ((rc = R.sync())) return rc;
        if (h.und_cnt[1] != 0) { gc_set_error("variant B: eviction times not final"); return GC_EHIP; }
        recs.push_back(RoundRec{U, U, maxmex, (long long)h.accepted, 0, passes});
        sweeps_total += passes;
    }
    gcl_finalize(d, gc_grid_for_waves(g->n, 8192), s);
    gcl_stat_reduce(d, s);
    GC_HIP(hipEventRecord(g->ev1, s));
    if (colors_out) GC_HIP(hipMemcpyAsync(colors_out, g->color, sizeof(int) * g->n, hipMemcpyDeviceToHost, s));
    if (cround_out) GC_HIP(hipMemcpyAsync(cround_out, g->cround, sizeof(int) * g->n, hipMemcpyDeviceToHost, s));
    if ((rc = R.sync())) return rc;
    if (st) {
        float ms = 0.f;
        GC_HIP(hipEventElapsedTime(&ms, g->ev0, g->ev1));
        st->device_ms = ms;
        st->rounds = (long long)recs.size();
        st->max_color = h.maxcolor;
        st->jp_sweeps = sweeps_total;
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
