// gc_priority.hip -- seeded priorities and the speculative first-fit mode (SURVEY.md §8b
// gc_color(..., priority, seed ...); BASELINE.json north_star: "Jones-Plassmann/Luby
// priority rounds on seeded hash priorities", "speculative first-fit coloring").
//
// The reference breaks every tie of its per-colour resolution by (deg, pos)
// (coloring.py:64: a stable sort by degree of a file-ordered group).  With
// gc_options.priority = 1 the same rounds run with rank (prio_hash(seed, v), pos) instead
// -- the tie-break fed with seeded priorities -- and the CPU oracle
// (oracle/gcolor_oracle.c, oracle_color_prio) computes the same function, so both sides
// are deterministic and comparable bit for bit.  The seed vertex and E1 keep the
// reference's argmax (deg, pos) rule; only the LFMIS order changes.
//
// Rank is static, so it lives in the row layout: every row lists its lower-rank entries
// first (nlow[v] of them) and every Jones-Plassmann sweep reads only those.  Switching the
// priority therefore re-partitions the rows once (gc_set_priority), in place (the column
// array keeps its address: shard views borrow it).  Hubs are a (deg, pos)-rank device --
// every hub ranks above every light vertex -- so a seeded run uses the row-scan path.
//
// gc_options.speculative = 1: speculative first-fit rounds with one-shot (Luby /
// Jones-Plassmann depth-1) conflict resolution.  Every uncoloured vertex proposes the mex
// of its coloured listed neighbours (0 if none), and keeps it iff no listed lower-rank
// neighbour proposed the same colour this round; everyone else retries next round.  One
// sweep per round instead of the LFMIS's chain of sweeps, no frontier push, no E1 (the
// lowest-rank uncoloured vertex always wins).  Not the reference's semantics -- the
// colour count is reported against it (tests/test_gpu_priority.py).
#include <string.h>

#include <algorithm>
#include <vector>

#include "gc_device.h"
#include "gc_engine.h"

namespace {

// per-round counter reset of a speculative round (one thread)
__global__ void k_spec_reset(GDev g, long long round) {
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
    c->bigw_cnt = 0;
    c->fsort_all = 1;
}

// one-shot resolution: v keeps its proposal iff no lower-rank listed entry (the nlow head
// of its row) proposed the same colour; every uncoloured vertex proposes, and candidates
// do not change during the pass, so the states written here never feed another decision.
// Heavy proposers (the heavy list k_propose built: deg > heavy_t) take a workgroup each and
// stop at their first same-candidate entry: a wave whose chunk held one walked its whole
// lower-rank part alone, the pass's long pole on R-MAT.
__global__ void __launch_bounds__(GC_BLOCK) k_spec_resolve(GDev g, GLists L) {
    DevCtl* c = g.ctl;
    {
        __shared__ unsigned s_hit;
        const long long hcnt = (long long)c->heavy_cnt;
        for (long long i = blockIdx.x; i < hcnt; i += gridDim.x) {
            const int v = L.heavy[i];
            const unsigned kv = g.k8[v];
            const unsigned c6 = gc_k8_cand(kv);
            const int cv = c6 == GC_K8_BIG ? g.cand[v] : (int)c6;
            const long long start = g.rp[v];
            const int dl = g.nlow[v];
            if (threadIdx.x == 0) s_hit = 0u;
            __syncthreads();
            for (int e0 = 0; e0 < dl; e0 += GC_SLOTS * GC_BLOCK) {
                unsigned hit = 0u;
#pragma unroll
                for (int k = 0; k < GC_SLOTS; ++k) {
                    const int e = e0 + k * GC_BLOCK + (int)threadIdx.x;
                    if (e < dl) {
                        const int u = g.col[start + e];
                        const unsigned ku = g.k8[u];
                        if (gc_k8_cand(ku) == c6 && (c6 != GC_K8_BIG || g.cand[u] == cv)) hit = 1u;
                    }
                }
                if (hit) s_hit = 1u;
                __syncthreads();
                const bool done = s_hit != 0u;
                __syncthreads();
                if (done) break;
            }
            if (threadIdx.x == 0) g.k8[v] = (unsigned char)((kv & ~3u) | (s_hit ? GC_JP_OUT : GC_JP_IN));
            __syncthreads();
        }
    }
    __shared__ long long s_start[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ unsigned s_flag[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ unsigned s_c6[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_cv[GC_WAVES_PER_BLOCK][GC_WAVE];
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    const int* __restrict__ list = L.F[c->cur];
    const long long cnt = (long long)c->fcnt[c->cur];
    const unsigned char* __restrict__ k8 = g.k8;
    const int vpw = gc_vpw(cnt, (long long)gridDim.x * GC_WAVES_PER_BLOCK);
    const long long nch = gc_nchunks(cnt, vpw);
    for (long long ch = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w; ch < nch;
         ch += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
        const long long idx = ch * vpw + lane;
        int v = (lane < vpw && idx < cnt) ? list[idx] : -1;
        if (v >= 0 && g.deg[v] > g.heavy_t) v = -1;  // in the heavy list (above)
        const unsigned kv = v >= 0 ? (unsigned)k8[v] : 0u;
        const unsigned c6 = v >= 0 ? gc_k8_cand(kv) : 0x100u;
        const int dl = v >= 0 ? g.nlow[v] : 0;
        s_start[w][lane] = v >= 0 ? g.rp[v] : 0;
        s_flag[w][lane] = 0;
        s_c6[w][lane] = c6;
        s_cv[w][lane] = c6 == GC_K8_BIG ? g.cand[v] : (int)c6;
        const int incl = gc_wave_incl_scan(dl);
        const int excl = incl - dl;
        const int total = __shfl(incl, GC_WAVE - 1, GC_WAVE);
        gc_wave_sync();
        gc_chunk_edges(
            g.col, s_start[w], excl, total, [&](int u) { return (unsigned)k8[u]; },
            [&](int o, int u, unsigned ku) {
                const unsigned oc = s_c6[w][o];
                if (gc_k8_cand(ku) != oc) return;
                if (oc == GC_K8_BIG && g.cand[u] != s_cv[w][o]) return;
                s_flag[w][o] = 1u;
            });
        gc_wave_sync();
        if (v >= 0) g.k8[v] = (unsigned char)((kv & ~3u) | (s_flag[w][lane] ? GC_JP_OUT : GC_JP_IN));
    }
}

// winners take their candidate (coloring.py:117-127)
__global__ void __launch_bounds__(GC_BLOCK) k_spec_commit(GDev g, GLists L, int* big) {
    DevCtl* c = g.ctl;
    __shared__ ull scratch[2 * GC_WAVES_PER_BLOCK];
    __shared__ long long s_start[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_cc[GC_WAVES_PER_BLOCK][GC_WAVE];
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
        const long long i = sidx * GC_WAVE + gc_lane();
        const int v = i < cnt ? list[i] : -1;
        const unsigned kv = v >= 0 ? (unsigned)g.k8[v] : 0u;
        const bool win = v >= 0 && gc_k8_state(kv) == GC_JP_IN;
        int cc = 0;
        if (win) {
            cc = gc_k8_cand(kv) == GC_K8_BIG ? g.cand[v] : (int)gc_k8_cand(kv);
            gc_commit_colour(g, v, cc);
            if (want_cround) g.cround[v] = round;
            lmaxc = cc > lmaxc ? cc : lmaxc;
            lacc++;
            lsum += (ull)g.deg[v];
        }
        // hub bitmaps (gc_hubs.hip): the winner's colour into every hub listing it
        if (g.hbits_w) gc_hub_push_wave(g, win, v, cc, s_start[w], s_cc[w], big, &c->bigw_cnt);
    }
    __syncthreads();
    gc_block_max(&c->maxcolor, lmaxc, (long long*)scratch);
    gc_block_add(&c->accepted, lacc, scratch);
    gc_stat_add(g, GC_K_COMMIT, lsum, lacc, scratch);
}

int sync_ctl(gc_graph* g) {
    GC_HIP(hipGetLastError());
    GC_HIP(hipMemcpyAsync(g->hctl, g->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, g->stream));
    GC_HIP(hipStreamSynchronize(g->stream));
    return GC_OK;
}

}  // namespace

// Rows re-partitioned for rank (key, pos): key = deg (priority 0, the reference) or
// prio_hash(seed, v) (priority 1).  In place: the partition goes to a scratch column array
// and is copied back, so rp / col keep their addresses.
int gc_set_priority(gc_graph* g, int prio, uint64_t seed) {
    if (prio != 0 && prio != 1) { gc_set_error("unknown priority %d", prio); return GC_EINVAL; }
    if (g->part_prio == prio && (prio == 0 || g->part_seed == seed)) return GC_OK;
    if (g->borrowed) { gc_set_error("a shard view cannot change the row partition"); return GC_EINVAL; }
    if (g->shard_refs > 0) {  // shards read col / nlow and the hub lists built under the (deg, pos) rank
        gc_set_error("%d shard(s) borrow this graph's (deg, pos) partition: destroy them before changing the priority",
                     g->shard_refs);
        return GC_EINVAL;
    }
    const hipStream_t s = g->stream;
    if (g->n > 0 && g->nnz > 0) {
        int* tmp = nullptr;
        if (gc_dmalloc((void**)&tmp, sizeof(int) * (size_t)g->nnz) != hipSuccess) {
            gc_set_error("allocation of the partition scratch (%lld entries) failed", g->nnz);
            return GC_ENOMEM;
        }
        if (g->hubflag) {  // the creation's hub flags follow the (deg, pos) row order: no longer valid
            hipStreamSynchronize(s);
            gc_dfree(g->hubflag);
            g->hubflag = nullptr;
            g->hubflag_t = -1;
        }
        int rc = gc_partition(g, g->col, tmp, prio, seed, &g->ctl->conflicts);
        hipError_t ec = hipSuccess;
        if (rc == GC_OK) ec = hipMemcpyAsync(g->col, tmp, sizeof(int) * (size_t)g->nnz, hipMemcpyDeviceToDevice, s);
        const hipError_t e = hipStreamSynchronize(s);
        gc_dfree(tmp);
        if (rc) return rc;
        if (ec != hipSuccess || e != hipSuccess || hipGetLastError() != hipSuccess) {
            gc_set_error("row re-partition failed");
            return GC_EHIP;
        }
        // the in-neighbour lists of an asymmetric graph are sets: their order is unaffected
    }
    g->part_prio = prio;
    g->part_seed = seed;
    g->bpart = prio == GC_PRIORITY_REF;  // the (deg, pos) partition also splits the low parts by degree
    return GC_OK;
}

// Speculative first-fit rounds (gc_options.speculative = 1) under the current rank.
int gc_color_speculative(gc_graph* g, const gc_options* opt, int32_t* colors_out, int32_t* cround_out, gc_stats* st) {
    const hipStream_t s = g->stream;
    GDev d = gc_view(g);
    const GLists L = gc_lists(g);
    // every uncoloured vertex proposes every round: hubs propose from pushed forbidden-colour
    // bitmaps (gc_hubs.hip) instead of re-reading their rows; the one-shot resolution needs
    // no hub JP
    int rc0 = gc_hubs_prepare(g, d);
    if (rc0) return rc0;
    d.hub_w = 0;
    d.tail_hmax = GC_TAIL_HMAX;
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
    // init + seed as the reference (coloring.py:12-35)
    gcl_init(d, g->seeds[0], gc_grid_for_waves(g->n), s);
    gcl_seed_prep(d, g->seeds[0], g->seeds[1], s);
    gcl_commit(d, L, GC_CM_INIT, 0, s);
    // every vertex counts as claimed: the re-sort then lists exactly the uncoloured ones
    GC_HIP(hipMemsetAsync(g->inF, 0xFF, sizeof(unsigned) * (size_t)((g->n + 63) / 32 + 2), s));
    std::vector<RoundRec> recs;
    int status = GC_OK, rc;
    long long fail_round = -1, fail_count = 0;
    const long long max_rounds = 4ll * g->n + 16;
    for (long long r = 0;; ++r) {
        if (r > max_rounds) { gc_set_error("round limit exceeded"); return GC_EROUNDS; }
        GC_LAUNCH(k_spec_reset, dim3(1), dim3(64), 0, s, d, r);
        gcl_fsort(d, L, g->fsum, s);
        if ((rc = sync_ctl(g))) return rc;
        const long long U = (long long)h.fcnt[0];
        if (U == 0) {
            recs.push_back(RoundRec{0, 0, -1, 0, 0, 0});
            break;
        }
        gcl_pack_c4(d, s);
        gcl_propose(d, L, s);
        gcl_propose_block(d, L, s);
        if ((rc = sync_ctl(g))) return rc;
        const long long maxmex = h.maxmex;
        if (h.kbound >= 0 && h.failcnt > 0) {  // state at the round start is returned
            recs.push_back(RoundRec{U, U, maxmex, 0, 0, 0});
            status = GC_FAILED;
            fail_round = r;
            fail_count = (long long)h.failcnt;
            break;
        }
        GC_LAUNCH(k_spec_resolve, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, d, L);
        GC_LAUNCH(k_spec_commit, dim3(GC_ROUND_GRID), dim3(GC_BLOCK), 0, s, d, L, g->ulist);
        if (d.hbits_w) gcl_hub_push_big(d, g->ulist, &g->ctl->bigw_cnt, s);
        if ((rc = sync_ctl(g))) return rc;
        recs.push_back(RoundRec{U, U, maxmex, (long long)h.accepted, 0, 1});
    }
    gcl_finalize(d, gc_grid_for_waves(g->n, 8192), s);
    gcl_stat_reduce(d, s);
    GC_HIP(hipEventRecord(g->ev1, s));
    if (colors_out) GC_HIP(hipMemcpyAsync(colors_out, g->color, sizeof(int) * g->n, hipMemcpyDeviceToHost, s));
    if (cround_out) GC_HIP(hipMemcpyAsync(cround_out, g->cround, sizeof(int) * g->n, hipMemcpyDeviceToHost, s));
    if ((rc = sync_ctl(g))) return rc;
    if (st) {
        float ms = 0.f;
        GC_HIP(hipEventElapsedTime(&ms, g->ev0, g->ev1));
        st->device_ms = ms;
        st->rounds = (long long)recs.size();
        st->max_color = h.maxcolor;
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
        st->k_bytes[GC_K_PROPOSE] = 24.0 * (double)h.nvert[GC_K_PROPOSE] + 8.0 * (double)h.sumdeg[GC_K_PROPOSE];
        st->k_bytes[GC_K_RESOLVE] = 24.0 * (double)h.nvert[GC_K_PROPOSE] + 12.0 * (double)h.sumdeg[GC_K_PROPOSE];
        st->k_bytes[GC_K_COMMIT] = 16.0 * (double)h.nvert[GC_K_COMMIT] + 8.0 * (double)h.sumdeg[GC_K_COMMIT];
    }
    return status;
}
