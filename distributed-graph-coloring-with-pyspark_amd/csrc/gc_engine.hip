// gc_engine.hip -- host engine: the round loop of graph_coloring (coloring.py:73-132) on
// one MI355X, plus validate_graph_coloring (coloring.py:149-162), behind the C-ABI.
//
// Every round is a fixed kernel schedule on one stream: propose -> resolve (JP sweeps
// until no vertex is undecided) -> commit+push.  The host only reads a 200-byte
// counter block back (pinned) at the few points where control flow depends on it.
#include <stdio.h>
#include <string.h>

#include <algorithm>

#include "gc_engine.h"

static thread_local std::string t_err;

void gc_set_error(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    t_err = buf;
}

extern "C" const char* gc_last_error(void) { return t_err.c_str(); }

extern "C" int gc_device_count(int32_t* count) {
    int c = 0;
    GC_HIP(hipGetDeviceCount(&c));
    *count = c;
    return GC_OK;
}

extern "C" int gc_set_device(int32_t device) {
    GC_HIP(hipSetDevice(device));
    return GC_OK;
}

GcDevView gc_view(const gc_graph* g) {
    GcDevView d;
    d.n = (int)g->n;
    d.nnz = g->nnz;
    d.rp = g->rp;
    d.col = g->col;
    d.deg = g->deg;
    d.trp = g->trp;
    d.tcol = g->tcol;
    d.color = g->color;
    d.cround = g->cround;
    d.key = g->key;
    d.jp = g->jp;
    d.inF = g->inF;
    d.ctl = g->ctl;
    return d;
}

template <typename T>
static int dalloc(T** p, size_t count) {
    if (count == 0) count = 1;
    hipError_t e = hipMalloc((void**)p, count * sizeof(T));
    if (e != hipSuccess) {
        gc_set_error("hipMalloc(%zu bytes) failed: %s", count * sizeof(T), hipGetErrorString(e));
        return GC_ENOMEM;
    }
    return GC_OK;
}

int gc_alloc_run_state(gc_graph* g) {
    if (g->has_run_state) return GC_OK;
    const size_t n = (size_t)g->n;
    int st = GC_OK;
#define A(p, c) if ((st = dalloc(&(p), (c))) != GC_OK) return st
    A(g->color, n);
    A(g->cround, n);
    A(g->key, n);
    A(g->jp, n);
    A(g->inF, (n + 63) / 32 + 2);
    A(g->F[0], n);
    A(g->F[1], n);
    A(g->heavy, n);
    A(g->wide, n);
    A(g->und[0], n);
    A(g->und[1], n);
    A(g->seeds[0], n);
    A(g->seeds[1], n);
    A(g->ulist, n);
    A(g->parent, n);
    A(g->best, n);
#undef A
    g->has_run_state = true;
    return GC_OK;
}

namespace {

// Optional per-launch event bracketing (gc_options.kernel_timing).
struct KTimer {
    gc_graph* g;
    bool on;
    gc_stats* st;
    std::vector<std::pair<int, size_t>> recs;  // (class, event index of start)
    size_t used = 0;
    hipEvent_t ev() {
        if (used >= g->evpool.size()) {
            hipEvent_t e;
            hipEventCreate(&e);
            g->evpool.push_back(e);
        }
        return g->evpool[used++];
    }
    void begin(int cls) {
        if (st) st->k_launches[cls]++;
        if (!on) return;
        recs.push_back({cls, used});
        hipEventRecord(ev(), g->stream);
    }
    void end() {
        if (!on) return;
        hipEventRecord(ev(), g->stream);
    }
    void collect() {
        if (!on || !st) return;
        for (auto& r : recs) {
            float ms = 0.f;
            hipEventElapsedTime(&ms, g->evpool[r.second], g->evpool[r.second + 1]);
            st->k_ms[r.first] += ms;
        }
    }
};

struct Run {
    gc_graph* g;
    const gc_options* opt;
    gc_stats* st;
    KTimer kt;
    GcDevView d;
    hipStream_t s;
    long long kbound;
    long long rounds = 0;

    int sync_ctl() {
        GC_HIP(hipMemcpyAsync(g->hctl, g->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, s));
        GC_HIP(hipStreamSynchronize(s));
        return GC_OK;
    }
    template <typename T>
    int zero(T* dev_field) {
        GC_HIP(hipMemsetAsync(dev_field, 0, sizeof(T), s));
        return GC_OK;
    }
    int set_i64(long long* dev_field, long long v) {
        // small values only: -1 via memset 0xFF
        if (v == -1) { GC_HIP(hipMemsetAsync(dev_field, 0xFF, sizeof(long long), s)); }
        else if (v == 0) { GC_HIP(hipMemsetAsync(dev_field, 0, sizeof(long long), s)); }
        else return GC_EINVAL;
        return GC_OK;
    }
    void record_round(long long U, long long F, long long maxmex, long long acc, long long seeds) {
        if (st && st->round_cap > rounds) {
            if (st->round_U) st->round_U[rounds] = U;
            if (st->round_F) st->round_F[rounds] = F;
            if (st->round_maxmex) st->round_maxmex[rounds] = maxmex;
            if (st->round_accepted) st->round_accepted[rounds] = acc;
            if (st->round_seeds) st->round_seeds[rounds] = seeds;
        }
        rounds++;
    }

    // commit the prepared seed lists (key/jp/inF already set) into frontier slot `dst`
    int commit_seeds(int dst, int round) {
        DevCtl& h = *g->hctl;
        int rc;
        if ((rc = sync_ctl())) return rc;
        const long long nl = (long long)h.seed_cnt[0], nh = (long long)h.seed_cnt[1];
        if (nl) {
            kt.begin(GC_K_COMMIT);
            gcl_commit_light(d, g->seeds[0], &g->ctl->seed_cnt[0], 0, g->F[dst], &g->ctl->fcnt[dst], round,
                             gc_grid_for_waves(nl), s);
            kt.end();
        }
        if (nh) {
            kt.begin(GC_K_COMMIT);
            gcl_commit_block(d, g->seeds[1], &g->ctl->seed_cnt[1], g->F[dst], &g->ctl->fcnt[dst], round,
                             (int)std::min<long long>(nh, 1024), s);
            kt.end();
        }
        return GC_OK;
    }

    int e1_reseed(int dst, int round, long long* nseeds) {
        int rc;
        if ((rc = zero(&g->ctl->list_cnt)) || (rc = zero(&g->ctl->seed_cnt[0])) || (rc = zero(&g->ctl->seed_cnt[1])))
            return rc;
        const int gridn = gc_grid_for_waves(g->n);
        kt.begin(GC_K_RESEED);
        gcl_unc_compact(d, g->ulist, &g->ctl->list_cnt, g->parent, g->best, gridn, s);
        kt.end();
        if ((rc = sync_ctl())) return rc;
        const long long L = (long long)g->hctl->list_cnt;
        kt.begin(GC_K_RESEED);
        gcl_cc_hook(d, g->ulist, &g->ctl->list_cnt, g->parent, gc_grid_for_waves(L), s);
        kt.end();
        kt.begin(GC_K_RESEED);
        gcl_cc_best(d, g->ulist, &g->ctl->list_cnt, g->parent, g->best, gc_grid_for_waves(L, 4096), s);
        kt.end();
        kt.begin(GC_K_RESEED);
        gcl_cc_seeds(d, g->ulist, &g->ctl->list_cnt, g->parent, g->best, g->seeds[0], g->seeds[1],
                     gc_grid_for_waves(L, 4096), s);
        kt.end();
        if ((rc = commit_seeds(dst, round))) return rc;
        *nseeds = (long long)(g->hctl->seed_cnt[0] + g->hctl->seed_cnt[1]);
        return GC_OK;
    }

    int go(int32_t* colors_out, int32_t* cround_out) {
        int rc;
        DevCtl& h = *g->hctl;
        GC_HIP(hipMemsetAsync(g->ctl, 0, sizeof(DevCtl), s));
        if ((rc = set_i64(&g->ctl->maxcolor, -1))) return rc;
        GC_HIP(hipEventRecord(g->ev0, s));
        // init + seed (coloring.py:74-76)
        kt.begin(GC_K_INIT);
        gcl_init(d, g->seeds[0], gc_grid_for_waves(g->n), s);
        kt.end();
        kt.begin(GC_K_INIT);
        gcl_seed_prep(d, g->seeds[0], g->seeds[1], s);
        kt.end();
        int cur = 0;
        if ((rc = commit_seeds(cur, 0))) return rc;
        if ((rc = sync_ctl())) return rc;
        long long U = (long long)h.uncolored - (h.seedkey ? 1 : 0);
        long long F = (long long)h.fcnt[cur];
        long long status = GC_OK;
        if (st) { st->fail_round = -1; st->fail_count = 0; }
        const long long max_rounds = 4ll * g->n + 16;
        for (long long r = 0;; ++r) {
            if (r > max_rounds) { gc_set_error("round limit exceeded"); return GC_EROUNDS; }
            if (U == 0) { record_round(0, 0, -1, 0, 0); break; }
            const int nxt = cur ^ 1;
            if (F == 0) {  // zero proposers: reference spins here (coloring.py:93-95)
                if (!opt->e1) { record_round(U, 0, -1, 0, 0); status = GC_STALLED; break; }
                if ((rc = zero(&g->ctl->fcnt[cur])) || (rc = zero(&g->ctl->accepted))) return rc;
                long long ns = 0;
                if ((rc = e1_reseed(cur, (int)r + 1, &ns))) return rc;
                if ((rc = sync_ctl())) return rc;
                record_round(U, 0, -1, 0, ns);
                if (st) st->reseeds += ns;
                U -= ns;
                F = (long long)h.fcnt[cur];
                continue;
            }
            // ---- propose ----
            if ((rc = zero(&g->ctl->heavy_cnt)) || (rc = zero(&g->ctl->wide_cnt)) || (rc = zero(&g->ctl->failcnt)) ||
                (rc = set_i64(&g->ctl->maxmex, -1)))
                return rc;
            kt.begin(GC_K_PROPOSE);
            gcl_propose_light(d, g->F[cur], &g->ctl->fcnt[cur], g->heavy, g->wide, kbound, gc_grid_for_waves(F), s);
            kt.end();
            if ((rc = sync_ctl())) return rc;
            const long long nh = (long long)h.heavy_cnt, nw = (long long)h.wide_cnt;
            if (nh + nw > 0) {
                long long words = (h.maxcolor + 2 + 31) / 32;
                words = std::max<long long>(1, std::min<long long>(words, 16384));
                kt.begin(GC_K_PROPOSE);
                gcl_propose_block(d, g->heavy, &g->ctl->heavy_cnt, g->wide, &g->ctl->wide_cnt, kbound, (int)words,
                                  (int)std::min<long long>(nh + nw, 4096), s);
                kt.end();
                if ((rc = sync_ctl())) return rc;
            }
            const long long maxmex = h.maxmex;
            if (kbound >= 0 && h.failcnt > 0) {  // coloring.py:104-108: state at round start
                record_round(U, F, maxmex, 0, 0);
                status = GC_FAILED;
                if (st) { st->fail_round = r; st->fail_count = (long long)h.failcnt; }
                break;
            }
            // ---- resolve: JP sweeps ----
            if ((rc = zero(&g->ctl->und_cnt[0]))) return rc;
            kt.begin(GC_K_RESOLVE);
            gcl_resolve_light(d, g->F[cur], &g->ctl->fcnt[cur], 1, g->und[0], &g->ctl->und_cnt[0], GC_K_RESOLVE,
                              gc_grid_for_waves(F), s);
            kt.end();
            if (nh) {
                kt.begin(GC_K_RESOLVE);
                gcl_resolve_block(d, g->heavy, &g->ctl->heavy_cnt, g->und[0], &g->ctl->und_cnt[0],
                                  (int)std::min<long long>(nh, 4096), s);
                kt.end();
            }
            if ((rc = sync_ctl())) return rc;
            int a = 0;
            while (h.und_cnt[a] > 0) {
                const long long nu = (long long)h.und_cnt[a];
                if ((rc = zero(&g->ctl->und_cnt[a ^ 1]))) return rc;
                kt.begin(GC_K_SWEEP);
                gcl_resolve_light(d, g->und[a], &g->ctl->und_cnt[a], 0, g->und[a ^ 1], &g->ctl->und_cnt[a ^ 1],
                                  GC_K_SWEEP, gc_grid_for_waves(nu), s);
                kt.end();
                if (st) st->jp_sweeps++;
                if ((rc = sync_ctl())) return rc;
                a ^= 1;
            }
            // ---- commit + frontier push ----
            if ((rc = zero(&g->ctl->fcnt[nxt])) || (rc = zero(&g->ctl->accepted))) return rc;
            kt.begin(GC_K_COMMIT);
            gcl_commit_light(d, g->F[cur], &g->ctl->fcnt[cur], 1, g->F[nxt], &g->ctl->fcnt[nxt], (int)r + 1,
                             gc_grid_for_waves(F), s);
            kt.end();
            if (nh) {
                kt.begin(GC_K_COMMIT);
                gcl_commit_block(d, g->heavy, &g->ctl->heavy_cnt, g->F[nxt], &g->ctl->fcnt[nxt], (int)r + 1,
                                 (int)std::min<long long>(nh, 1024), s);
                kt.end();
            }
            if ((rc = sync_ctl())) return rc;
            const long long acc = (long long)h.accepted;
            record_round(U, F, maxmex, acc, 0);
            U -= acc;
            cur = nxt;
            F = (long long)h.fcnt[cur];
        }
        GC_HIP(hipEventRecord(g->ev1, s));
        if (colors_out) GC_HIP(hipMemcpyAsync(colors_out, g->color, sizeof(int) * g->n, hipMemcpyDeviceToHost, s));
        if (cround_out) GC_HIP(hipMemcpyAsync(cround_out, g->cround, sizeof(int) * g->n, hipMemcpyDeviceToHost, s));
        if ((rc = sync_ctl())) return rc;
        if (st) {
            float ms = 0.f;
            GC_HIP(hipEventElapsedTime(&ms, g->ev0, g->ev1));
            st->device_ms = ms;
            st->rounds = rounds;
            st->max_color = h.maxcolor;
            // SURVEY.md §8d algorithmic bytes per kernel class
            st->k_bytes[GC_K_PROPOSE] = 24.0 * (double)h.nvert[1] + 8.0 * (double)h.sumdeg[1];
            st->k_bytes[GC_K_RESOLVE] = 24.0 * (double)h.nvert[2] + 12.0 * (double)h.sumdeg[2];
            st->k_bytes[GC_K_COMMIT] = 16.0 * (double)h.nvert[4] + 8.0 * (double)h.sumdeg[4];
            kt.collect();
        }
        return (int)status;
    }
};

}  // namespace

extern "C" int gc_color(gc_graph* g, const gc_options* opt, int32_t* colors_out, int32_t* cround_out,
                        gc_stats* stats) {
    if (!g || !opt) { gc_set_error("gc_color: null argument"); return GC_EINVAL; }
    if (opt->variant != GC_VARIANT_A) {
        gc_set_error("gc_color: variant %d not available on this build", opt->variant);
        return GC_EINVAL;
    }
    GC_HIP(hipSetDevice(g->device));
    int rc = gc_alloc_run_state(g);
    if (rc) return rc;
    if (stats) {
        // keep caller's round buffers, clear outputs
        gc_stats keep = *stats;
        memset(stats, 0, sizeof(*stats));
        stats->round_cap = keep.round_cap;
        stats->round_U = keep.round_U;
        stats->round_F = keep.round_F;
        stats->round_maxmex = keep.round_maxmex;
        stats->round_accepted = keep.round_accepted;
        stats->round_seeds = keep.round_seeds;
        stats->max_color = -1;
    }
    Run run{g, opt, stats, KTimer{g, opt->kernel_timing != 0, stats, {}, 0}, gc_view(g), g->stream,
            opt->num_colors, 0};
    rc = run.go(colors_out, cround_out);
    if (rc < 0) return rc;
    if (stats && stats->round_cap < run.rounds && (stats->round_U || stats->round_F)) {
        gc_set_error("round buffers too small: %lld rounds", run.rounds);
        return GC_EROUNDS;
    }
    return rc;
}

extern "C" int gc_validate(gc_graph* g, const int32_t* colors, int64_t* uncolored, int64_t* conflicts) {
    if (!g) { gc_set_error("gc_validate: null graph"); return GC_EINVAL; }
    GC_HIP(hipSetDevice(g->device));
    int rc = gc_alloc_run_state(g);
    if (rc) return rc;
    const int* src = g->color;
    if (colors) {
        if (!g->vcolors && (rc = dalloc(&g->vcolors, (size_t)g->n))) return rc;
        GC_HIP(hipMemcpyAsync(g->vcolors, colors, sizeof(int) * g->n, hipMemcpyHostToDevice, g->stream));
        src = g->vcolors;
    }
    GC_HIP(hipMemsetAsync(&g->ctl->uncolored, 0, sizeof(ull), g->stream));
    GC_HIP(hipMemsetAsync(&g->ctl->conflicts, 0, sizeof(ull), g->stream));
    gcl_validate(gc_view(g), src, gc_grid_for_waves(g->n), g->stream);
    GC_HIP(hipGetLastError());
    GC_HIP(hipMemcpyAsync(g->hctl, g->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, g->stream));
    GC_HIP(hipStreamSynchronize(g->stream));
    if (uncolored) *uncolored = (int64_t)g->hctl->uncolored;
    if (conflicts) *conflicts = (int64_t)g->hctl->conflicts;
    return GC_OK;
}
