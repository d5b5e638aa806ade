// gc_shard.hip -- one rank's share of a multi-GPU colouring, C-ABI.
//
// Every rank holds the whole CSR (a gc_graph handle; R-MAT-28 is ~36 GB of a GPU's
// 288 GB) and owns a contiguous vertex range [lo, hi).  A shard is a view of that graph
// with its own run state and a rank-local in-neighbour CSR (the owned rows' targets), so
// the single-GPU round kernels run unchanged on the rank's own frontier.  A round is cut
// at its grid-wide seams (coloring.py:73-132):
//   propose  -> publish (v, candidate) of the rank's proposers      (coloring.py:44-54)
//   resolve, JP sweeps -> publish (v, IN|OUT) of decided ones       (coloring.py:56-70)
// The caller (gcolor_amd/shard.py) all-gathers them over RCCL -- as int64 deltas
// (vertex << 32 | value) into gc_shard_apply, or as every rank's slice of the proposal
// bytes (gc_shard_get_slice / put_slices) when most vertices changed -- so after the last
// sweep seam every rank holds every proposer's final state and gc_shard_finish colours
// all winners (coloring.py:114-127) with no further exchange.  Because the conflict
// resolution is the lexicographically-first MIS under the global rank (deg, pos), the
// result does not depend on the partition: it is bit-identical to gc_color on one GPU.
//
// The phase calls that return counts synchronise (the caller needs them for the exchange);
// apply / get_slice / put_slices only enqueue.  gc_shard_set_stream puts the shard on the
// caller's stream (torch's, where the RCCL collectives run), so a seam -- phase, copy into
// the send buffer, all-gather, apply -- is ordered on one stream with no host wait inside.
#include <string.h>

#include <algorithm>
#include <chrono>

#include "gc_engine.h"

struct gc_shard {
    gc_graph v;  // borrowed CSR + own in-neighbour CSR + own run state
    long long lo = 0, hi = 0;
    // Hub forbidden-colour bitmaps (gc_hubs.hip) for the proposals of the heavy vertices:
    // the hub lists (hid, hin) are the parent graph's, built once at gc_shard_create; the
    // bitmaps are this rank's replica, kept current by pushes from every winner, the rank's
    // own (k_commit) and the others' (k_shard_list_commit / k_shard_scan_commit).
    gc_graph* parent = nullptr;
    gc_graph* owner = nullptr;  // the graph whose rows this shard borrows (its shard_refs counts us)
    unsigned* hbits = nullptr;
    int hub_w = 0;
    long long nhub = 0;
    // Replicated hubs (the default; GC_SHARD_HUBS=0 turns them off): every rank holds the
    // hub JP state of EVERY hub (deg > the parent's hub threshold) and runs it on the
    // replicated light states, so hubs are proposed, resolved and committed by every rank
    // alike and never travel.  A rank lists every frontier hub (its own through its
    // in-neighbour pushes, the others' through hseen, gc_shard_hub_claim); the hub JP starts
    // once every rank's lights have converged (gc_shard_start_hubs) and runs to its end with
    // no exchange, as the one-GPU engine's hub sweeps do (gc_hubs.hip).
    bool repl = false;
    int tail_hmax = 4 * GC_TAIL_HMAX_HUB;  // hubs the one-workgroup tail sweeps take (GC_SHARD_TAIL_HMAX)
    unsigned *hk = nullptr, *hkill = nullptr;
    int *hcur = nullptr, *hpc = nullptr, *hrow = nullptr, *hlen = nullptr, *hkcnt = nullptr, *hseen = nullptr;
};

// the shard's kernel arguments: its own view plus the parent's hub lists and its bitmaps
static GDev shard_view(gc_shard* sh) {
    GDev d = gc_view(&sh->v);
    const gc_graph* p = sh->parent;
    if (sh->hbits && p && p->nhub == sh->nhub && p->hub_w == sh->hub_w) {
        d.hbits_w = sh->hub_w;
        d.hbits = sh->hbits;
        d.hb_stride = sh->nhub;
        d.hid = p->hid;
        d.hin_rp = p->hin_rp;
        d.hin_col = p->hin_col;
        if (sh->repl) {  // the parent's read-only hub lists, this shard's hub JP state
            d.heavy_t = p->hub_t;
            d.hub_w = sh->hub_w;
            d.hub_v = p->hub_v;
            d.hlow_rp = p->hlow_rp;
            d.hlow_col = p->hlow_col;
            d.hlowb[0] = p->hlow_col;
            d.hk = sh->hk;
            d.hkill = sh->hkill;
            d.hcur = sh->hcur;
            d.hpc = sh->hpc;
            d.hrow = sh->hrow;
            d.hlen = sh->hlen;
            d.hkcnt = sh->hkcnt;
            d.hub_scan = 1;  // the resumable row scan (no per-round row copies to replicate)
            d.hprep = 0;
            d.hub_long = GC_HUB_LONG;
            d.tail_hmax = sh->tail_hmax;  // the async hub JP (gc_shard_start_hubs_async) leans on the tail
            d.hub_repl = 1;
            d.own_lo = sh->lo;
            d.own_hi = sh->hi;
            d.hseen = sh->hseen;
            d.nhub_repl = sh->nhub;
        }
    }
    return d;
}

static void shard_free_hubs(gc_shard* sh) {
    void* ptrs[] = {sh->hbits, sh->hk, sh->hkill, sh->hcur, sh->hpc, sh->hrow, sh->hlen, sh->hkcnt, sh->hseen};
    for (void* p : ptrs)
        if (p) gc_dfree(p);
    sh->hbits = sh->hk = sh->hkill = nullptr;
    sh->hcur = sh->hpc = sh->hrow = sh->hlen = sh->hkcnt = sh->hseen = nullptr;
    sh->repl = false;
}

// the shard's hub arrays: the bitmaps, and with replicated hubs the hub JP state
static int shard_alloc_hubs(gc_shard* sh) {
    const size_t H = (size_t)sh->nhub;
    if (gc_dmalloc((void**)&sh->hbits, sizeof(unsigned) * H * (size_t)sh->hub_w) != hipSuccess) {
        sh->hbits = nullptr;
        gc_set_error("hipMalloc of the shard's hub bitmaps failed");
        return GC_ENOMEM;
    }
    if (!sh->repl) return GC_OK;
    void** arrs[] = {(void**)&sh->hk, (void**)&sh->hkill, (void**)&sh->hcur, (void**)&sh->hpc,
                     (void**)&sh->hrow, (void**)&sh->hlen, (void**)&sh->hkcnt, (void**)&sh->hseen};
    for (void** a : arrs) {
        if (gc_dmalloc(a, 4 * H) != hipSuccess) {
            *a = nullptr;
            gc_set_error("hipMalloc of the shard's hub state failed");
            return GC_ENOMEM;
        }
    }
    return GC_OK;
}

static int shard_sync(gc_shard* sh) {
    gc_graph* g = &sh->v;
    GC_HIP(hipGetLastError());
    GC_HIP(hipMemcpyAsync(g->hctl, g->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, g->stream));
    GC_HIP(hipStreamSynchronize(g->stream));
    if (g->hctl->loop_err == GC_LERR_LIST) {
        gc_set_error("shard: a work-list append passed the list's capacity (round %lld)", g->hctl->round);
        return GC_EHIP;
    }
    return GC_OK;
}

static GLists shard_lists(gc_shard* sh, int64_t* delta) {
    GLists L = gc_lists(&sh->v);
    L.delta = reinterpret_cast<long long*>(delta);
    return L;
}

extern "C" int gc_shard_create(gc_graph* g, int64_t lo, int64_t hi, gc_shard** out) {
    if (!g || !out) { gc_set_error("gc_shard_create: null argument"); return GC_EINVAL; }
    if (lo < 0 || hi < lo || hi > g->n) { gc_set_error("gc_shard_create: bad range [%lld, %lld)", (long long)lo, (long long)hi); return GC_EINVAL; }
    GC_HIP(hipSetDevice(g->device));
    // GC_PREP_TIMING=1: host-side phase times on stderr (each phase ends in a synchronisation)
    const bool timing = getenv("GC_PREP_TIMING") != nullptr;
    auto tmark = [&, t = std::chrono::steady_clock::now()](const char* what) mutable {
        if (!timing) return;
        hipDeviceSynchronize();
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[gc shard] %-14s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    };
    int rc0 = gc_set_priority(g, GC_PRIORITY_REF, 0);  // shards run the reference's (deg, pos) rank
    if (rc0) return rc0;
    tmark("priority");
    gc_shard* sh = new gc_shard();
    gc_graph& v = sh->v;
    v.device = g->device;
    v.n = g->n;
    v.nnz = g->nnz;
    v.maxdeg = g->maxdeg;
    v.flags = g->flags & ~GC_GRAPH_SYMMETRIC;
    v.borrowed = true;
    v.rp = g->rp;
    v.col = g->col;
    v.deg = g->deg;
    v.nlow = g->nlow;
    sh->lo = lo;
    sh->hi = hi;
    if (getenv("GC_SHARD_TAIL_HMAX")) sh->tail_hmax = std::max(0, atoi(getenv("GC_SHARD_TAIL_HMAX")));
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&v.stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipEventCreate(&v.ev0)) != hipSuccess || (e = hipEventCreate(&v.ev1)) != hipSuccess ||
        (e = gc_dmalloc((void**)&v.ctl, sizeof(DevCtl))) != hipSuccess ||
        (e = gc_hmalloc((void**)&v.hctl, sizeof(DevCtl))) != hipSuccess) {
        gc_set_error("shard allocation failed: %s", hipGetErrorString(e));
        gc_free_all(&v);
        delete sh;
        return GC_ENOMEM;
    }
    // symmetric graphs: the rows' entries in [lo, hi), entry-parallel over the parent's tiling
    // (GC_SHARD_INROWS=wave: round 4's row-per-wave kernels)
    const char* ir = getenv("GC_SHARD_INROWS");
    int rc = !(g->flags & GC_GRAPH_SYMMETRIC) ? gc_build_in_csr(&v, lo, hi)
             : (ir && strcmp(ir, "wave") == 0)  ? gc_build_in_csr_sym(&v, lo, hi)
                                                : gc_filter_rows_sym(g, &v, lo, hi);
    tmark("in-rows");
    if (!rc) rc = gc_alloc_run_state(&v);
    tmark("run state");
    if (!rc) {  // hub lists on the parent (once), a bitmap replica (+ hub JP state) for this shard
        GDev pd = gc_view(g);
        rc = gc_hubs_prepare(g, pd);
        tmark("hub index");
        const char* env = getenv("GC_SHARD_HUBS");
        const bool want_repl = !(env && *env && atoi(env) == 0);
        if (!rc && g->nhub > 0 && want_repl && g->hub_t >= 0) {  // every deg > hub_t vertex is a hub
            sh->parent = g;
            sh->hub_w = g->hub_w;
            sh->nhub = g->nhub;
            sh->repl = true;
            rc = shard_alloc_hubs(sh);
        } else if (!rc && g->nhub > 0 && v.maxdeg > GC_HEAVY_T && g->hub_t <= GC_HEAVY_T) {
            // bitmaps only: the heavy proposers (deg > GC_HEAVY_T) are hubs
            sh->parent = g;
            sh->hub_w = g->hub_w;
            sh->nhub = g->nhub;
            rc = shard_alloc_hubs(sh);
        }
    }
    tmark("hub replica");
    // without replicated hubs the shards resolve heavy vertices by row scans
    if (!rc && !sh->repl && g->maxdeg > GC_HEAVY_T) rc = gc_alloc_heavy_pending(&v);
    if (rc) {
        shard_free_hubs(sh);
        std::string keep = gc_last_error();
        gc_free_all(&v);
        delete sh;
        gc_set_error("%s", keep.c_str());
        return rc;
    }
    sh->owner = g;
    g->shard_refs++;
    *out = sh;
    return GC_OK;
}

extern "C" void gc_shard_destroy(gc_shard* sh) {
    if (!sh) return;
    gc_graph* owner = sh->owner;
    gc_free_all(&sh->v);
    shard_free_hubs(sh);
    delete sh;
    if (owner && --owner->shard_refs == 0 && owner->destroy_pending) gc_graph_destroy(owner);
}

// init + seed on the replicated state (coloring.py:74-76); the seeds push into the
// rank's own in-neighbours.  U is global (replicated), F is this rank's frontier.
extern "C" int gc_shard_begin(gc_shard* sh, int64_t num_colors, int32_t track_rounds, int64_t* U_out, int64_t* F_out) {
    if (!sh) { gc_set_error("null shard"); return GC_EINVAL; }
    gc_graph* g = &sh->v;
    if (sh->owner && (sh->owner->part_prio != GC_PRIORITY_REF ||
                      (sh->parent && (sh->parent->nhub != sh->nhub || sh->parent->hub_prio != GC_PRIORITY_REF)))) {
        gc_set_error("gc_shard_begin: the parent graph's row partition or hub lists changed under the shard");
        return GC_EINVAL;
    }
    GC_HIP(hipSetDevice(g->device));
    DevCtl& h = *g->hctl;
    memset(&h, 0, sizeof(DevCtl));
    h.kbound = num_colors;
    h.e1 = 1;
    h.rcap = g->rcap;
    h.maxmex = -1;
    h.maxcolor = -1;
    h.fail_round = -1;
    h.want_cround = track_rounds ? 1 : 0;
    GC_HIP(hipMemcpyAsync(g->ctl, &h, sizeof(DevCtl), hipMemcpyHostToDevice, g->stream));
    if (sh->hbits)
        GC_HIP(hipMemsetAsync(sh->hbits, 0, sizeof(unsigned) * (size_t)sh->nhub * (size_t)sh->hub_w, g->stream));
    if (sh->repl) {  // hk: k_init; hcur / hpc: every proposal
        for (int* a : {sh->hrow, sh->hlen, sh->hkcnt, sh->hseen})
            GC_HIP(hipMemsetAsync(a, 0, 4 * (size_t)sh->nhub, g->stream));
        GC_HIP(hipMemsetAsync(sh->hkill, 0, 4 * (size_t)sh->nhub, g->stream));
    }
    const GDev d = shard_view(sh);
    const GLists L = shard_lists(sh, nullptr);
    gcl_init(d, g->seeds[0], gc_grid_for_waves(g->n), g->stream);
    gcl_seed_prep(d, g->seeds[0], g->seeds[1], g->stream);
    gcl_commit(d, L, GC_CM_INIT, 0, g->stream);
    gcl_shard_hub_claim(d, L, 0, g->stream);  // other ranks' hubs next to a seed
    int rc = shard_sync(sh);
    if (rc) return rc;
    if (U_out) *U_out = (int64_t)h.uncolored - (h.seedkey ? 1 : 0);
    if (F_out) *F_out = (int64_t)h.fcnt[h.cur];
    return GC_OK;
}

// propose on the rank's frontier; delta = (v, candidate) per proposer.
// stats: [0] deltas written, [1] frontier size, [2] max candidate (-1), [3] #candidates >= k
extern "C" int gc_shard_propose(gc_shard* sh, int64_t round, int64_t* delta, int64_t cap, int64_t* stats) {
    if (!sh || !delta || !stats) { gc_set_error("null argument"); return GC_EINVAL; }
    gc_graph* g = &sh->v;
    if (cap < sh->hi - sh->lo) { gc_set_error("delta capacity %lld < owned range", (long long)cap); return GC_EINVAL; }
    GC_HIP(hipSetDevice(g->device));
    const GDev d = shard_view(sh);
    const GLists L = shard_lists(sh, delta);
    gcl_shard_reset(d, round, g->stream);
    gcl_fsort(d, L, g->fsum, g->stream);  // big rounds: the rank's frontier in vertex order
    gcl_pack_c4(d, g->stream);
    gcl_propose(d, L, g->stream);
    gcl_propose_block(d, L, g->stream);
    gcl_delta_cand(d, L, g->stream);
    int rc = shard_sync(sh);
    if (rc) return rc;
    const DevCtl& h = *g->hctl;
    stats[0] = (int64_t)(sh->repl ? h.dcnt : h.fcnt[h.cur]);
    stats[1] = (int64_t)(h.fcnt[h.cur] - h.xhub_cnt);
    stats[2] = h.maxmex;
    stats[3] = (int64_t)h.failcnt;
    return GC_OK;
}

// Run the shard's kernels on the caller's stream from now on (e.g. torch's current stream,
// so the RCCL collectives that move the seams are ordered with them).
extern "C" int gc_shard_set_stream(gc_shard* sh, void* stream) {
    if (!sh) { gc_set_error("null shard"); return GC_EINVAL; }
    gc_graph* g = &sh->v;
    GC_HIP(hipSetDevice(g->device));
    if (stream) {  // a stream of another GPU would run the shard's kernels on the wrong device
        hipDevice_t sd = -1;
        GC_HIP(hipStreamGetDevice(reinterpret_cast<hipStream_t>(stream), &sd));
        if ((int)sd != g->device) {
            gc_set_error("gc_shard_set_stream: the stream belongs to device %d, the graph to device %d", (int)sd, g->device);
            return GC_EINVAL;
        }
    }
    GC_HIP(hipStreamSynchronize(g->stream));
    if (g->own_stream && g->stream) GC_HIP(hipStreamDestroy(g->stream));
    g->stream = reinterpret_cast<hipStream_t>(stream);
    g->own_stream = false;
    return GC_OK;
}

// Asynchronous phases (nothing waits; the counts go into the seam's header, gc_shard_pack):
// propose on the rank's frontier with (v, candidate) deltas, and JP sweeps i .. i+count-1
// with (v, IN|OUT) deltas (delta == null: a slice seam follows, no deltas written).
extern "C" int gc_shard_propose_async(gc_shard* sh, int64_t round, int64_t* delta, int64_t cap) {
    if (!sh || !delta) { gc_set_error("null argument"); return GC_EINVAL; }
    gc_graph* g = &sh->v;
    if (cap < sh->hi - sh->lo) { gc_set_error("delta capacity %lld < owned range", (long long)cap); return GC_EINVAL; }
    GC_HIP(hipSetDevice(g->device));
    const GDev d = shard_view(sh);
    const GLists L = shard_lists(sh, delta);
    gcl_shard_reset(d, round, g->stream);
    gcl_fsort(d, L, g->fsum, g->stream);
    gcl_pack_c4(d, g->stream);
    gcl_propose(d, L, g->stream);
    // no heavy (deg > heavy_t) or wide (mex >= 64, so deg >= 64) proposer possible: no
    // k_propose_block launch (meshes: one launch of host time per round, as in gc_color)
    if (g->maxdeg > d.heavy_t || g->maxdeg >= 64) gcl_propose_block(d, L, g->stream);
    gcl_delta_cand(d, L, g->stream);
    GC_HIP(hipGetLastError());
    return GC_OK;
}

extern "C" int gc_shard_sweep_async(gc_shard* sh, int32_t i, int32_t count, int64_t* delta, int64_t cap) {
    if (!sh || i < 0 || count < 1) { gc_set_error("bad argument"); return GC_EINVAL; }
    gc_graph* g = &sh->v;
    if (delta && cap < sh->hi - sh->lo) { gc_set_error("delta capacity %lld < owned range", (long long)cap); return GC_EINVAL; }
    GC_HIP(hipSetDevice(g->device));
    const GDev d = shard_view(sh);
    const GLists L = shard_lists(sh, delta);
    GC_HIP(hipMemsetAsync(&g->ctl->dcnt, 0, sizeof(ull), g->stream));
    for (int j = i; j < i + count; ++j) {
        if (j == 0) gcl_resolve(d, L, g->stream);
        else gcl_sweep(d, L, j, g->stream);
    }
    GC_HIP(hipGetLastError());
    return GC_OK;
}

// The seam's send buffer on the device: header words (the rank's round scalars) + up to cap
// deltas (kind GC_KIND_CAND after propose, GC_KIND_STATE after sweeps whose last list slot is
// `slot`); send holds GC_SEAM_HDR + cap int64.  delta == null: header only (slice seams
// put the proposal-byte slice after it with gc_shard_get_slice).
extern "C" int gc_shard_pack(gc_shard* sh, int32_t kind, int32_t slot, const int64_t* delta, int64_t* send,
                             int64_t cap) {
    if (!sh || !send || cap < 0 || slot < 0 || slot > 2) { gc_set_error("bad argument"); return GC_EINVAL; }
    gc_graph* g = &sh->v;
    GC_HIP(hipSetDevice(g->device));
    gcl_shard_pack(shard_view(sh), kind, slot, reinterpret_cast<const long long*>(delta),
                   reinterpret_cast<long long*>(send), delta ? cap : 0, g->stream);
    GC_HIP(hipGetLastError());
    return GC_OK;
}

// apply every rank's deltas of one kind to the vertices this rank does not own (enqueued,
// no wait); IN states are also listed as the round's remote winners (gc_shard_finish)
extern "C" int gc_shard_apply(gc_shard* sh, int32_t kind, const int64_t* recv, int64_t count, int64_t round) {
    if (!sh) { gc_set_error("null shard"); return GC_EINVAL; }
    if (kind < GC_KIND_CAND || kind > GC_KIND_COLOUR) { gc_set_error("bad delta kind %d", kind); return GC_EINVAL; }
    gc_graph* g = &sh->v;
    GC_HIP(hipSetDevice(g->device));
    if (count > 0 && !recv) { gc_set_error("null delta buffer"); return GC_EINVAL; }
    gcl_apply(shard_view(sh), kind, reinterpret_cast<const long long*>(recv), count, sh->lo, sh->hi, (int)round + 1,
              kind == GC_KIND_STATE ? g->parent : nullptr, g->stream);
    GC_HIP(hipGetLastError());
    return GC_OK;
}

// A fused propose seam's apply (the first JP sweep is enqueued behind it before the host has
// read any header): applied only if every rank's header allows it, else the shard halts with
// GC_H_SEAM, so the sweep behind it does nothing; gc_shard_clear_halt(GC_H_SEAM) undoes it.
extern "C" int gc_shard_apply_checked(gc_shard* sh, int32_t kind, const int64_t* recv, int64_t count, int64_t round,
                                      int64_t hdr_stride) {
    if (!sh || hdr_stride <= GC_SEAM_HDR || (count > 0 && !recv)) { gc_set_error("bad argument"); return GC_EINVAL; }
    gc_graph* g = &sh->v;
    GC_HIP(hipSetDevice(g->device));
    gcl_apply(shard_view(sh), kind, reinterpret_cast<const long long*>(recv), count, sh->lo, sh->hi, (int)round + 1,
              kind == GC_KIND_STATE ? g->parent : nullptr, g->stream, hdr_stride);
    GC_HIP(hipGetLastError());
    return GC_OK;
}

extern "C" int gc_shard_clear_halt(gc_shard* sh, int32_t code) {
    if (!sh) { gc_set_error("null shard"); return GC_EINVAL; }
    gc_graph* g = &sh->v;
    GC_HIP(hipSetDevice(g->device));
    gcl_shard_clear_halt(shard_view(sh), code, g->stream);
    GC_HIP(hipGetLastError());
    return GC_OK;
}

// JP sweeps i, i+1, ..., i+count-1 over the rank's lists (i = 0 is the first sweep over
// the frontier; later sweeps run over the undecided); the rank's later sweeps can decide
// vertices whose lower-rank neighbours are its own, so several run between two
// exchanges.  delta = (v, IN|OUT) of every vertex decided, or null when the seam will
// move slices instead.  stats: [0] deltas, [1] still undecided on this rank
extern "C" int gc_shard_sweep(gc_shard* sh, int32_t i, int32_t count, int64_t* delta, int64_t cap, int64_t* stats) {
    if (!sh || !stats || i < 0 || count < 1) { gc_set_error("bad argument"); return GC_EINVAL; }
    gc_graph* g = &sh->v;
    if (delta && cap < sh->hi - sh->lo) { gc_set_error("delta capacity %lld < owned range", (long long)cap); return GC_EINVAL; }
    GC_HIP(hipSetDevice(g->device));
    const GDev d = shard_view(sh);
    const GLists L = shard_lists(sh, delta);
    GC_HIP(hipMemsetAsync(&g->ctl->dcnt, 0, sizeof(ull), g->stream));
    for (int j = i; j < i + count; ++j) {
        if (j == 0) gcl_resolve(d, L, g->stream);
        else gcl_sweep(d, L, j, g->stream);
    }
    int rc = shard_sync(sh);
    if (rc) return rc;
    const DevCtl& h = *g->hctl;
    const int last = (i + count - 1) % 3;
    stats[0] = (int64_t)h.dcnt;
    stats[1] = (int64_t)(h.und_cnt[last] + h.undh_cnt[last]) +
               (sh->repl && h.hub_start == GC_HUB_NOT_STARTED ? (int64_t)h.heavy_cnt : 0);
    return GC_OK;
}

// Replicated hubs: the number of hubs (0: hubs, if any, are resolved through the exchange).
extern "C" int gc_shard_hub_count(gc_shard* sh, int64_t* nhub) {
    if (!sh || !nhub) { gc_set_error("null argument"); return GC_EINVAL; }
    *nhub = sh->repl ? (int64_t)sh->nhub : 0;
    return GC_OK;
}

static int hub_sweeps_to_end(gc_shard* sh, int j0, int64_t* sweeps_out);

// Replicated hubs, once every rank's lights are decided (every rank's sweep seam reported no
// undecided light): start the hub JP at sweep i and run it to its end on this rank (every
// rank runs the same sweeps on the same state, so no exchange).  from_slices: a slice seam
// moved light states this round, so the other ranks' light winners flag their hubs here
// (delta seams flagged them in gc_shard_apply).  sweeps_out: sweeps run (i, i+1, ...).
extern "C" int gc_shard_start_hubs(gc_shard* sh, int32_t i, int32_t from_slices, int64_t* sweeps_out) {
    if (!sh || i < 1) { gc_set_error("bad argument"); return GC_EINVAL; }
    gc_graph* g = &sh->v;
    if (sweeps_out) *sweeps_out = 0;
    if (!sh->repl) return GC_OK;
    GC_HIP(hipSetDevice(g->device));
    const GDev d = shard_view(sh);
    if (from_slices) gcl_shard_hub_flags(d, sh->lo, sh->hi, g->stream);
    GC_HIP(hipMemsetAsync(&g->ctl->lights_hold, 0, sizeof(int), g->stream));
    return hub_sweeps_to_end(sh, i, sweeps_out);
}

// The asynchronous form: the hubs' first `grid` sweeps (i, i+1, ...) on the full grid, then
// the one-workgroup tail (k_sweep_tail) runs the rest of the chain while the lists stay
// within its limits.  Nothing waits: gc_shard_finish_async(check = 1) verifies on the device
// that the hub JP converged (else the round halts with GC_H_SWEEPS, reported in the next
// propose seam's header, and gc_shard_resume_hubs finishes it).  Every rank runs the same
// sweeps on the same replicated state, so every rank halts alike.
extern "C" int gc_shard_start_hubs_async(gc_shard* sh, int32_t i, int32_t from_slices, int32_t grid) {
    if (!sh || i < 1 || grid < 1) { gc_set_error("bad argument"); return GC_EINVAL; }
    gc_graph* g = &sh->v;
    if (!sh->repl) return GC_OK;
    GC_HIP(hipSetDevice(g->device));
    const GDev d = shard_view(sh);
    const GLists L = shard_lists(sh, nullptr);
    if (from_slices) gcl_shard_hub_flags(d, sh->lo, sh->hi, g->stream);
    GC_HIP(hipMemsetAsync(&g->ctl->lights_hold, 0, sizeof(int), g->stream));
    for (int k = 0; k < grid; ++k) gcl_sweep(d, L, i + k, g->stream);
    gcl_sweep_tail(d, L, i + grid - 1, g->stream);
    GC_HIP(hipGetLastError());
    return GC_OK;
}

// After a finish that halted (the previous propose seam's header carried -GC_H_SWEEPS on
// every rank): clear the halt and run the hub sweeps from the first one not yet run to
// their end (host-paced, as gc_shard_start_hubs); then the caller enqueues the finish again.
extern "C" int gc_shard_resume_hubs(gc_shard* sh, int64_t* sweeps_out) {
    if (!sh) { gc_set_error("null shard"); return GC_EINVAL; }
    gc_graph* g = &sh->v;
    if (sweeps_out) *sweeps_out = 0;
    GC_HIP(hipSetDevice(g->device));
    int rc = shard_sync(sh);
    if (rc) return rc;
    if (g->hctl->halt != GC_H_SWEEPS) { gc_set_error("gc_shard_resume_hubs: the shard is not halted for sweeps"); return GC_EINVAL; }
    const long long j = g->hctl->sweeps_enq + 1;
    GC_HIP(hipMemsetAsync(&g->ctl->halt, 0, sizeof(int), g->stream));
    return hub_sweeps_to_end(sh, (int)j, sweeps_out);
}

// hub sweeps j0, j0+1, ... in batches, host-paced, until the lists are empty
static int hub_sweeps_to_end(gc_shard* sh, int j0, int64_t* sweeps_out) {
    gc_graph* g = &sh->v;
    const GDev d = shard_view(sh);
    const GLists L = shard_lists(sh, nullptr);
    const int i = j0;
    const int batch = 8;  // sweeps past the end find no work and return at once
    long long j = i;
    for (;;) {
        for (int k = 0; k < batch; ++k) gcl_sweep(d, L, (int)(j + k), g->stream);
        j += batch;
        int rc = shard_sync(sh);
        if (rc) return rc;
        const DevCtl& h = *g->hctl;
        const int last = (int)((j - 1) % 3);
        if ((h.und_cnt[last] | h.undh_cnt[last]) == 0 && h.hub_start != GC_HUB_NOT_STARTED) break;
        if (j - i > 4 * (long long)sh->nhub + 64) {
            gc_set_error("gc_shard_start_hubs: the hub sweeps did not converge");
            return GC_EINVAL;
        }
    }
    if (sweeps_out) *sweeps_out = (int64_t)(j - i);
    const long long tl = j - 1;  // the last sweep run: what a checked finish looks at
    GC_HIP(hipMemcpy(&g->ctl->tail_last, &tl, sizeof(long long), hipMemcpyHostToDevice));
    return GC_OK;
}

// Dense form of the propose / sweep seams when most vertices changed: the rank's slice
// [lo, hi) of the proposal bytes k8 (cand6 << 2 | JP state) instead of 8-byte deltas.
extern "C" int gc_shard_get_slice(gc_shard* sh, uint8_t* dst) {
    if (!sh || !dst) { gc_set_error("null argument"); return GC_EINVAL; }
    gc_graph* g = &sh->v;
    GC_HIP(hipSetDevice(g->device));
    if (sh->hi > sh->lo)
        GC_HIP(hipMemcpyAsync(dst, g->k8 + sh->lo, (size_t)(sh->hi - sh->lo), hipMemcpyDeviceToDevice, g->stream));
    return GC_OK;
}

// src holds `parts` slices of `stride` bytes; slice p covers [starts[p], starts[p]+lens[p])
// (host arrays).  Every slice but the rank's own is copied into k8.
extern "C" int gc_shard_put_slices(gc_shard* sh, const uint8_t* src, int64_t stride, const int64_t* starts,
                                   const int64_t* lens, int32_t parts) {
    if (!sh || !src || !starts || !lens) { gc_set_error("null argument"); return GC_EINVAL; }
    gc_graph* g = &sh->v;
    GC_HIP(hipSetDevice(g->device));
    for (int p = 0; p < parts; ++p) {
        if (lens[p] <= 0 || (starts[p] == sh->lo && lens[p] == sh->hi - sh->lo)) continue;  // own slice
        if (starts[p] < 0 || starts[p] + lens[p] > g->n || lens[p] > stride) { gc_set_error("bad slice %d", p); return GC_EINVAL; }
        GC_HIP(hipMemcpyAsync(g->k8 + starts[p], src + (size_t)p * (size_t)stride, (size_t)lens[p],
                              hipMemcpyDeviceToDevice, g->stream));
    }
    return GC_OK;
}

// End of the round (coloring.py:114-127): colour every winner -- the rank's own through
// its frontier (losers stay in it), the other ranks' from the IN state deltas received
// this round (from_deltas: every sweep seam of the round moved deltas) or read off the
// replicated proposal bytes (a slice seam moved some states without deltas) -- push them
// into this rank's in-neighbours and make that frontier current.
// acc_out: winners of ALL ranks (the same on every rank); F_out: the rank's new frontier.
static int shard_finish_enqueue(gc_shard* sh, int32_t from_deltas, int32_t check) {
    gc_graph* g = &sh->v;
    GC_HIP(hipSetDevice(g->device));
    const GDev d = shard_view(sh);
    const GLists L = shard_lists(sh, nullptr);
    gcl_commit(d, L, GC_CM_SHARD, check ? GC_SHARD_CHECK : 0, g->stream);
    if (from_deltas) gcl_shard_list_commit(d, L, g->parent, g->ulist, g->stream);
    else gcl_shard_scan_commit(d, L, sh->lo, sh->hi, g->ulist, g->stream);
    if (d.hbits_w) gcl_hub_push_big(d, g->ulist, &g->ctl->list_cnt, g->stream);  // the other ranks' winners
    gcl_shard_flip(d, g->stream);
    gcl_shard_hub_claim(d, L, 0, g->stream);  // the other ranks' hubs next to this round's winners
    GC_HIP(hipGetLastError());
    return GC_OK;
}

extern "C" int gc_shard_finish(gc_shard* sh, int64_t round, int32_t from_deltas, int64_t* acc_out, int64_t* F_out) {
    if (!sh) { gc_set_error("null shard"); return GC_EINVAL; }
    gc_graph* g = &sh->v;
    int rc = shard_finish_enqueue(sh, from_deltas, 0);
    if (!rc) rc = shard_sync(sh);
    if (rc) return rc;
    if (acc_out) *acc_out = (int64_t)g->hctl->accepted;
    if (F_out) *F_out = (int64_t)g->hctl->fcnt[g->hctl->cur];
    (void)round;
    return GC_OK;
}

// The same, only enqueued: the winners' count reaches the host in the next propose seam's
// header (k_shard_pack, word 4).  check = 1: the hub JP ran asynchronously
// (gc_shard_start_hubs_async); the commit first verifies on the device that it converged.
extern "C" int gc_shard_finish_async(gc_shard* sh, int64_t round, int32_t from_deltas, int32_t check) {
    if (!sh) { gc_set_error("null shard"); return GC_EINVAL; }
    (void)round;
    return shard_finish_enqueue(sh, from_deltas, check);
}

// E1 on the replicated state (identical seeds on every rank), seeds pushed into the
// rank's own in-neighbours.
extern "C" int gc_shard_reseed(gc_shard* sh, int64_t round, int64_t* nseeds, int64_t* F_out) {
    if (!sh) { gc_set_error("null shard"); return GC_EINVAL; }
    gc_graph* g = &sh->v;
    GC_HIP(hipSetDevice(g->device));
    const GDev d = shard_view(sh);
    const GLists L = shard_lists(sh, nullptr);
    gcl_shard_reset(d, round, g->stream);
    gcl_unc_compact(d, g->ulist, &g->ctl->list_cnt, g->parent, g->best, gc_grid_for_waves(g->n), g->stream);
    int rc = shard_sync(sh);
    if (rc) return rc;
    const long long Lc = (long long)g->hctl->list_cnt;
    gcl_cc_hook(d, g->ulist, &g->ctl->list_cnt, g->parent, gc_grid_for_waves(Lc), g->stream);
    gcl_cc_best(d, g->ulist, &g->ctl->list_cnt, g->parent, g->best, gc_grid_for_waves(Lc, 4096), g->stream);
    gcl_cc_seeds(d, g->ulist, &g->ctl->list_cnt, g->parent, g->best, g->seeds[0], g->seeds[1],
                 gc_grid_for_waves(Lc, 4096), g->stream);
    gcl_commit(d, L, GC_CM_RESEED, 0, g->stream);
    gcl_shard_hub_claim(d, L, 0, g->stream);
    if ((rc = shard_sync(sh))) return rc;
    if (nseeds) *nseeds = (int64_t)(g->hctl->seed_cnt[0] + g->hctl->seed_cnt[1]);
    if (F_out) *F_out = (int64_t)g->hctl->fcnt[g->hctl->cur];
    return GC_OK;
}

// final colours (every rank holds all of them) and optionally the round of colouring
// The replicated colours (and rounds) into caller DEVICE buffers, and the rank's own frontier
// (its F[cur] without the other ranks' replicated hubs) into front_dev (capacity hi - lo):
// what gc_color_resume needs to finish the colouring on the one-GPU engine.
extern "C" int gc_shard_export(gc_shard* sh, int32_t* colors_dev, int32_t* cround_dev, int32_t* front_dev,
                               int64_t* nfront) {
    if (!sh || !colors_dev || !front_dev || !nfront) { gc_set_error("gc_shard_export: null argument"); return GC_EINVAL; }
    gc_graph* g = &sh->v;
    GC_HIP(hipSetDevice(g->device));
    const GDev d = shard_view(sh);
    const GLists L = shard_lists(sh, nullptr);
    gcl_finalize(d, gc_grid_for_waves(g->n, 8192), g->stream);
    GC_HIP(hipMemcpyAsync(colors_dev, g->color, sizeof(int) * g->n, hipMemcpyDeviceToDevice, g->stream));
    if (cround_dev) GC_HIP(hipMemcpyAsync(cround_dev, g->cround, sizeof(int) * g->n, hipMemcpyDeviceToDevice, g->stream));
    GC_HIP(hipMemsetAsync(&g->ctl->list_cnt, 0, sizeof(ull), g->stream));
    gcl_shard_own_front(d, L, sh->lo, sh->hi, front_dev, &g->ctl->list_cnt, g->stream);
    int rc = shard_sync(sh);
    if (rc) return rc;
    *nfront = (int64_t)g->hctl->list_cnt;
    GC_HIP(hipMemsetAsync(&g->ctl->list_cnt, 0, sizeof(ull), g->stream));
    return GC_OK;
}

extern "C" int gc_shard_colors(gc_shard* sh, int32_t* colors_out, int32_t* cround_out) {
    if (!sh) { gc_set_error("null shard"); return GC_EINVAL; }
    gc_graph* g = &sh->v;
    GC_HIP(hipSetDevice(g->device));
    gcl_finalize(shard_view(sh), gc_grid_for_waves(g->n, 8192), g->stream);
    if (colors_out) GC_HIP(hipMemcpyAsync(colors_out, g->color, sizeof(int) * g->n, hipMemcpyDeviceToHost, g->stream));
    if (cround_out) GC_HIP(hipMemcpyAsync(cround_out, g->cround, sizeof(int) * g->n, hipMemcpyDeviceToHost, g->stream));
    return shard_sync(sh);
}
