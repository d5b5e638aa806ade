// gc_engine.hip -- host engine: the round loop of graph_coloring (coloring.py:73-132) on
// one MI355X, plus validate_graph_coloring (coloring.py:149-162), behind the C-ABI.
//
// The host never waits on a round.  It enqueues batches of rounds -- [frontier re-sort],
// pack_c4, propose, propose_block, resolve, S sweeps, commit, close -- and every kernel
// takes its counts from the device control block; k_close ends each round on the device
// (record, counter reset, termination).  The host keeps one batch in flight (1-4 rounds),
// reads a pinned snapshot of the control block per batch, and only steps in for the
// rare events the device cannot finish alone: an E1 re-seed (zero proposers, uncoloured
// vertices left), a round whose Jones-Plassmann depth exceeded the S sweeps enqueued
// (more sweeps, then the commit again), a full round-record buffer.
#include <chrono>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>

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

thread_local long long gc_tl_launches = 0;

static thread_local hipStream_t t_input_stream = nullptr;
static thread_local bool t_input_stream_set = false;

extern "C" int gc_set_input_stream(void* stream, int32_t enable) {
    t_input_stream = (hipStream_t)stream;
    t_input_stream_set = enable != 0;
    return GC_OK;
}

int gc_order_after_inputs(hipStream_t s) {
    if (!t_input_stream_set) {
        GC_HIP(hipDeviceSynchronize());
        return GC_OK;
    }
    hipEvent_t ev;
    GC_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    hipError_t e = hipEventRecord(ev, t_input_stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(s, ev, 0);
    hipEventDestroy(ev);  // released once the wait completes
    GC_HIP(e);
    return GC_OK;
}

GDev gc_view(const gc_graph* g) {
    GDev d;
    d.n = (int)g->n;
    d.nnz = g->nnz;
    // GC_TEST_LIST_CAP (tests only): a smaller capacity for the staged list appends, so that a
    // colouring hits the overflow path (reported GC_EHIP, pipeline halted) on a small graph
    d.list_cap = g->n;
    if (const char* e = getenv("GC_TEST_LIST_CAP")) {
        const long long c = atoll(e);
        if (c >= 0 && c < d.list_cap) d.list_cap = c;
    }
    d.rp = g->rp;
    d.col = g->col;
    d.deg = g->deg;
    d.nlow = g->nlow;
    d.trp = g->trp;
    d.tcol = g->tcol;
    d.color = g->color;
    d.cround = g->cround;
    d.cand = g->cand;
    d.c8 = g->c8;
    d.c4 = g->c4;
    d.k8 = g->k8;
    d.inF = g->inF;
    d.mark = g->mark;
    d.ctl = g->ctl;
    d.lcur = g->lcur;
    d.bstat = g->bstat;
    d.accs = nullptr;  // the single-GPU variant-A engine turns it on (Run)
    d.bigrow = getenv("GC_BIGROW") ? atoi(getenv("GC_BIGROW")) : GC_BIGROW;  // env: tests / tuning
    d.big_rows = !((g->flags & GC_GRAPH_SYMMETRIC) && 2 * g->maxdeg <= d.bigrow);
    d.claim_direct = getenv("GC_CLAIM_DIRECT") ? atoi(getenv("GC_CLAIM_DIRECT")) : 0;
    d.hpl = g->hpl;
    d.hplc = g->hplc;
    d.hub_repl = 0;
    d.own_lo = 0;
    d.own_hi = g->n;
    d.hseen = nullptr;
    d.nhub_repl = 0;
    d.heavy_t = GC_HEAVY_T;
    d.hub_w = 0;
    d.hbits_w = 0;
    d.hub_long = 0;
    d.tail_hmax = GC_TAIL_HMAX;
    d.b_resident = 0;
    d.b_watch = 0;
    d.b_awin = 8;
    d.b_refskip = 0;
    d.a_watch = getenv("GC_A_WATCH") ? atoi(getenv("GC_A_WATCH")) : 0;
    d.tail_lmax = getenv("GC_TAIL_LMAX") ? atoi(getenv("GC_TAIL_LMAX")) : GC_TAIL_MAX;
    d.tail_nw = getenv("GC_TAIL_WAVES") ? atoi(getenv("GC_TAIL_WAVES")) : GC_TAIL_WAVES;
    d.tail_nw = d.tail_nw >= 16 ? 16 : (d.tail_nw >= 8 ? 8 : 4);
    d.heavy_wg = 0;
    d.hch_rp = nullptr;
    d.hch_own = nullptr;
    d.hkcnt = nullptr;
    d.nhch = 0;
    d.hch_mul = 1;
    d.hprep = 0;
    d.hcore = d.core_hub = nullptr;
    d.core_bits = nullptr;
    d.core_wcnt = nullptr;
    d.core_cap = 0;
    d.nhub_core = 0;
    d.core_iters = 0;
    d.hub_scan = 0;
    d.hk = nullptr;
    d.hid = nullptr;
    d.hub_v = nullptr;
    d.hin_rp = nullptr;
    d.hin_col = nullptr;
    d.hbits = nullptr;
    d.hb_stride = 0;
    d.hkill = nullptr;
    d.hlow_rp = nullptr;
    d.hlow_col = nullptr;
    d.hcur = nullptr;
    d.hpc = nullptr;
    d.hpend[0] = d.hpend[1] = nullptr;
    d.hrow = d.hlen = nullptr;
    d.hlowb[0] = d.hlowb[1] = d.hlowb[2] = nullptr;
    return d;
}

GLists gc_lists(const gc_graph* g) {
    GLists L;
    L.F[0] = g->F[0];
    L.F[1] = g->F[1];
    L.heavy = g->heavy;
    L.wide = g->wide;
    for (int k = 0; k < 3; ++k) {
        L.undL[k] = g->undL[k];
        L.undH[k] = g->undH[k];
    }
    L.seeds[0] = g->seeds[0];
    L.seeds[1] = g->seeds[1];
    L.bigw = g->bigw;
    L.rec = g->rec;
    L.delta = nullptr;
    return L;
}

template <typename T>
static int dalloc(T** p, size_t count) {
    if (count == 0) count = 1;
    hipError_t e = gc_dmalloc((void**)p, count * sizeof(T));
    if (e != hipSuccess) {
        gc_set_error("gc_dmalloc(%zu bytes) failed: %s", count * sizeof(T), hipGetErrorString(e));
        return GC_ENOMEM;
    }
    return GC_OK;
}

static const long long kRoundCap = 4096;

// The hubs-off heavy JP (a workgroup per heavy vertex, gc_jp_sweep) keeps, per round, the
// entries of a heavy vertex's lower-rank part that can still block it (same candidate,
// undecided) at hpl[rp[v] ..]: its later sweeps read those instead of the whole part
// (R-MAT hubs: ~10^5 entries).  Only seeded ranks, shards and hubs-off runs take that path.
int gc_alloc_heavy_pending(gc_graph* g) {
    if (g->hpl) return GC_OK;
    int st = dalloc(&g->hpl, (size_t)std::max<long long>(g->nnz, 1));
    if (st == GC_OK) st = dalloc(&g->hplc, (size_t)std::max<long long>(g->n, 1));
    return st;
}

int gc_alloc_run_state(gc_graph* g) {
    if (g->has_run_state) return GC_OK;
    const size_t n = (size_t)g->n;
    int st = GC_OK;
#define A(p, c) if ((st = dalloc(&(p), (c))) != GC_OK) return st
    A(g->color, n);
    A(g->cround, n);
    A(g->cand, n);
    A(g->lcur, n);
    A(g->bstat, (size_t)GC_STAT_SLOTS * 16);
    A(g->accs, (size_t)GC_ACC_SLOTS + GC_TICK_WORDS);  // + k_commit_big's arrival tickets
    A(g->c8, n);
    A(g->c4, n / 8 + 2);
    A(g->k8, n);
    A(g->inF, (n + 63) / 32 + 2);
    A(g->mark, n + 64);
    A(g->F[0], n);
    A(g->F[1], n);
    A(g->heavy, n);
    A(g->wide, n);
    for (int k = 0; k < 3; ++k) {
        A(g->undL[k], n);
        A(g->undH[k], n);
    }
    A(g->seeds[0], n);
    A(g->seeds[1], n);
    A(g->bigw, n);
    A(g->ulist, n);
    A(g->parent, n);
    A(g->best, n);
    A(g->rec, (size_t)kRoundCap);
    A(g->fsum, (size_t)gcl_fsort_blocks(g->n) + 1);
#undef A
    GC_HIP(gc_hmalloc((void**)&g->hsnap, 2 * sizeof(DevCtl)));
    GC_HIP(hipHostGetDevicePointer((void**)&g->hsnap_dev, g->hsnap, 0));
    GC_HIP(hipEventCreateWithFlags(&g->evsnap[0], hipEventDisableTiming));
    GC_HIP(hipEventCreateWithFlags(&g->evsnap[1], hipEventDisableTiming));
    g->rcap = kRoundCap;
    g->has_run_state = true;
    return GC_OK;
}

namespace {

// Optional event timing of kernel classes (gc_options.kernel_timing).  A RUN of
// consecutive launches of one timed class (a round's JP sweeps, say) is bracketed by ONE
// event pair: bracketing every launch cost ~5 us per launch in gaps (R-MAT-24: ~10k sweep
// launches per colouring).  The run's time includes the launch gaps inside it, so the
// class time is an upper bound of its kernels' busy time.  Runs are closed at every host
// synchronisation and at the end of every round, so no host wait is ever inside one.
// (KTimer: gc_engine.h, shared with variant B)

struct ResumeArgs {
    const int* colors;  // device int32[n], -1 uncoloured
    const int* cround;  // device int32[n] or null
    const int* front;   // device int32[nf]: the uncoloured vertices with a coloured listed neighbour
    long long nf;
    long long round0;   // rounds already run
};

struct Run {
    gc_graph* g;
    const gc_options* opt;
    gc_stats* st;
    KTimer kt;
    GDev d;
    GLists L;
    hipStream_t s;
    std::vector<RoundRec> recs;  // drained round records
    long long drained = 0;       // absolute index of the first record not yet drained
    bool debug = getenv("GC_DEBUG") != nullptr;
    bool resort_hint = false;    // enqueue the frontier re-sort kernels (last snapshot's frontier >= n/256)
    bool c4_hint = true;         // enqueue k_pack_c4 (last snapshot's frontier >= n/64, colours < 14)
    const int batch_max = getenv("GC_BATCH_MAX") ? atoi(getenv("GC_BATCH_MAX")) : 4;
    // k_sweep_loop's grid: one workgroup per CU (all resident: its grid barrier needs it).
    // Off unless GC_SWEEP_LOOP=1: it cuts the sweep launches ~2.5x but measured slower
    // (R-MAT-26 588 -> 610 ms, C2 8.0 -> 12.2 ms: a grid barrier costs about a launch, and
    // the resident grid has a quarter of the waves for the latency-bound sweeps)
    int loop_grid = 0;
    // k_sweep_async (the default with the hub JP's resumable scan, or with no heavy vertex):
    // the JP chain after the first sweep in ONE launch on a resident grid (CUs x blocks per
    // CU), instead of full-grid sweeps plus the one-workgroup tail.  GC_ASYNC=0 turns it off;
    // GC_ASYNC_BPC (blocks per CU, default 2, capped by the occupancy), GC_ASYNC_BUDGET_US
    // (per launch, default 20000: a launch past it hands its rest to host sweeps).
    int async_grid = 0;
    int async_par = 0;
    long long async_budget = 0;
    // (round 4 measured the big rounds -- frontier >= n/256 -- on the full-grid sweeps and the
    // one-workgroup tail instead: R-MAT-24 +6.1%, R-MAT-26 +5.0%, profiles/r04/g; the
    // asynchronous JP stays on in every round)
    void init_async() {
        const char* e = getenv("GC_ASYNC");
        if (e && atoi(e) == 0) return;
        // Only with the hub JP's resumable scan (R-MAT and the like).  Graphs with no hub keep
        // the full-grid sweeps and the one-workgroup tail: round 4 measured the asynchronous
        // JP on them (bit-exact, profiles/r04/b) at C2 12.1 -> 18.8 ms and mesh 512^3 111.6 ->
        // 111.6 ms (profiles/r04/c), so it stays off there -- their JP chains are short (C2:
        // 15 rounds, meshes depth 1) and a resident grid has a quarter of the full grid's waves.
        if (!d.hub_w || !d.hub_scan || d.heavy_wg || L.delta) return;
        int cus = 0, rate_khz = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, g->device) != hipSuccess || cus <= 0)
            return;
        if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, g->device) != hipSuccess || rate_khz <= 0)
            return;
        int bpc = getenv("GC_ASYNC_BPC") ? atoi(getenv("GC_ASYNC_BPC")) : 2;
        const int occ = gcl_sweep_async_resident(d, g->stream);  // resident workgroups per CU, measured (gc_residency_probe)
        if (occ <= 0) return;
        bpc = std::max(1, std::min(bpc, occ));
        const long long us = getenv("GC_ASYNC_BUDGET_US") ? atoll(getenv("GC_ASYNC_BUDGET_US")) : 20000;
        async_budget = std::max(1ll, us) * (long long)rate_khz / 1000;
        async_grid = cus * bpc;
        // GC_ASYNC_WG (tests): fewer workgroups, so each wave holds long hub and light lists
        if (getenv("GC_ASYNC_WG") && atoi(getenv("GC_ASYNC_WG")) > 0) async_grid = std::min(async_grid, atoi(getenv("GC_ASYNC_WG")));
        // the hub core (gc_core.hip): its buffers once per graph; GC_HUB_CORE=0 off
        if (!d.hub_repl && gc_core_prepare(g, d) == GC_OK) core_on = d.core_cap > 0;
    }
    // The hub core: a build is attempted (gcl_core_build, before the next batch) once a
    // snapshot's next frontier is at most twice the core's capacity and 20% below the last
    // attempt's; k_hub_core runs ahead of every k_sweep_async once a snapshot shows it READY.
    bool core_on = false, core_ready = false, core_pending = false;
    long long core_try_f = -1;  // frontier at the last build attempt (-1: none yet)
    // k_hub_core only while the last snapshot's frontier is at least GC_HUB_CORE_MINF (1024): below
    // it a round has ~100 hub proposers, ~2 JP passes, and k_sweep_async alone is as fast
    long long core_f = 0;
    const long long core_min_f = getenv("GC_HUB_CORE_MINF") ? atoll(getenv("GC_HUB_CORE_MINF")) : 1024;
    const bool core_debug = getenv("GC_CORE_DEBUG") != nullptr;
    void core_check(const DevCtl& x) {
        core_f = (long long)x.fcnt[x.cur];
        if (!core_on || core_ready) return;
        if (x.core_state == GC_CORE_READY) {
            core_ready = true;
            if (core_debug) fprintf(stderr, "[gc core] ready at round %lld: %d hubs\n", x.round, x.core_n);
            return;
        }
        const long long f = (long long)x.fcnt[x.cur];
        if (f > 0 && f <= 2ll * d.core_cap && (core_try_f < 0 || f * 5 <= core_try_f * 4)) {
            if (core_debug)
                fprintf(stderr, "[gc core] build attempt before round %lld (frontier %lld; last attempt: state %d, %llu "
                                "uncoloured hubs)\n", x.round, f, x.core_state, x.core_cnt);
            core_pending = true;
            core_try_f = f;
        }
    }
    void init_loop() {
        const char* e = getenv("GC_SWEEP_LOOP");
        if (!e || atoi(e) <= 0) return;
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, g->device) != hipSuccess || cus <= 0)
            return;
        const char* w = getenv("GC_LOOP_WG");
        loop_grid = w && atoi(w) > 0 ? std::min(atoi(w), cus) : cus;
    }
    // k_propose_block has no work unless some vertex can be heavy or wide: skip its launch
    // (meshes: ~5 us of a ~80 us round)
    bool need_pblock() const { return g->maxdeg > d.heavy_t || g->maxdeg >= 64; }  // heavy_t is final once hubs are set
    // Small rounds propose their hubs and wide lights inside k_propose<1> (a wave each) and
    // skip the k_propose_block launch (round 4: R-MAT-24 158.7 -> 155.4 ms, R-MAT-26 429.4 ->
    // 429.0, profiles/r04/g; GC_INLINE_PB=0 turns it off).  Needs the hub bitmaps (heavy ==
    // hub) and lights narrow enough for k_propose's 2048-bit window; the bitmaps must cover
    // every colour the enqueued rounds can reach (maxcolor grows by at most one a round: the
    // last snapshot's maxcolor plus a margin of the rounds in flight).
    bool inline_pb = !(getenv("GC_INLINE_PB") && atoi(getenv("GC_INLINE_PB")) == 0);
    long long maxc_hint = 1ll << 40;  // the last snapshot's maxcolor (none yet: no inlining; a resumed colouring's colours are unknown here)
    // GC_TEST_INL_MARGIN (tests only) replaces the margin, so a test can make the inlined
    // proposals outrun a small bitmap and exercise the fallback of color_impl
    const long long inl_margin = getenv("GC_TEST_INL_MARGIN") ? atoll(getenv("GC_TEST_INL_MARGIN")) : 2 + 4ll * batch_max + 16;
    bool inline_now() const {
        return inline_pb && !resort_hint && d.hbits_w && !d.hub_repl && d.heavy_t < 2048 &&
               maxc_hint + inl_margin <= 32ll * d.hbits_w;
    }
    // Fused commits (k_commit<1>) make the next round's proposals themselves, so a round
    // after one runs no k_propose: low-degree graphs (no heavy or wide proposer, no hubs),
    // small rounds (the big-round frontier rebuild and nibble mirror stay unfused).
    // GC_FUSE=0 turns it off (A/B measurements).
    bool fuse_ok = false;
    bool proposed = false;  // the next round's proposals were made by the last commit enqueued
    bool fuse_now() const { return fuse_ok && !resort_hint && !c4_hint; }

    int sync_ctl() {
        kt.close();
        GC_HIP(hipMemcpyAsync(g->hctl, g->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, s));
        GC_HIP(hipStreamSynchronize(s));
        if (async_grid > 0) {
            // k_sweep_async launches that were enqueued behind a halt returned at once, so the
            // launch parity no longer says which counter slot the last launch that RAN zeroed:
            // start both slots (and the parity) afresh before anything else is enqueued
            GC_HIP(hipMemsetAsync(g->ctl->async_done, 0, sizeof(g->ctl->async_done), s));
            GC_HIP(hipMemsetAsync(g->ctl->async_abort, 0, sizeof(g->ctl->async_abort), s));
            async_par = 0;
        }
        if (d.accs)  // k_commit_big's tickets: a launch cut short by a halt may have left arrivals
            GC_HIP(hipMemsetAsync(d.accs + GC_ACC_SLOTS, 0, sizeof(ull) * GC_TICK_WORDS, s));
        if (debug) {
            const DevCtl& h = *g->hctl;
            fprintf(stderr, "[gc] halt=%d round=%lld U=%lld cur=%d fcnt=%llu/%llu und=%llu/%llu/%llu undh=%llu/%llu/%llu "
                            "sweeps=%lld enq=%lld maxdepth=%lld\n",
                    h.halt, h.round, h.U, h.cur, h.fcnt[0], h.fcnt[1], h.und_cnt[0], h.und_cnt[1], h.und_cnt[2],
                    h.undh_cnt[0], h.undh_cnt[1], h.undh_cnt[2], h.sweeps, h.sweeps_enq, h.maxdepth);
        }
        return GC_OK;
    }
    int clear_halt() {
        GC_HIP(hipMemsetAsync(&g->ctl->halt, 0, sizeof(int), s));
        return GC_OK;
    }
    // copy the device records [drained, round) out and restart the device buffer
    int drain_records() {
        kt.close();
        const long long r = g->hctl->round;
        const long long cnt = r - drained;
        if (cnt > 0) {
            const size_t off = recs.size();
            recs.resize(off + (size_t)cnt);
            GC_HIP(hipMemcpyAsync(recs.data() + off, g->rec, sizeof(RoundRec) * (size_t)cnt, hipMemcpyDeviceToHost,
                                  s));
        }
        drained = r;
        GC_HIP(hipMemcpyAsync(&g->ctl->rbase, &g->hctl->round, sizeof(long long), hipMemcpyHostToDevice, s));
        GC_HIP(hipStreamSynchronize(s));
        return GC_OK;
    }

    // big = the host also enqueues the big-round frontier build (k_pull, k_front_*): the
    // device then decides per round (gc_big_on) whether the commit pushes or marks.
    void launch_commit(int mode, int nsweeps, bool fuse = false) {
        const int big = mode == GC_CM_ROUND && resort_hint && !fuse;
        // no sweeps enqueued and >= 16 rounds so far all decided by their first sweep (meshes):
        // no tail kernel either; a round that needs more makes the commit ask for sweeps
        // (GC_H_SWEEPS), which come with the tail (nsweeps -1 tells k_commit it did not run)
        const bool tail = mode == GC_CM_ROUND && (nsweeps > 0 || !skip_tail);
        if (tail && async_grid > 0) {  // the rest of the JP chain: one asynchronous launch
            kt.begin(GC_K_SWEEP);
            if (core_ready && core_f >= core_min_f) gcl_hub_core(d, L, nsweeps, async_par, s);  // decides the hubs when it can
            gcl_sweep_async(d, L, nsweeps, async_par, async_budget, async_grid, s, resort_hint ? 1 : 0);
            async_par ^= 1;
            kt.end();
        } else if (tail && loop_grid > 0) {  // the middle of the JP chain: one resident-grid launch
            kt.begin(GC_K_SWEEP);
            gcl_sweep_loop(d, L, nsweeps, loop_grid, s);
            kt.end();
        }
        if (tail && async_grid == 0) {
            kt.begin(GC_K_SWEEP);
            gcl_sweep_tail(d, L, nsweeps, s);
            kt.end();
        }
        // the commit's last workgroup closes the round unless k_pull / the big-round frontier
        // rebuild / k_commit_big must run between the commit and the close
        // (graphs with big rows keep a k_close launch: closing in k_commit_big's last workgroup
        // measured slower, R-MAT-24 172.7 -> 176.8 ms, profiles/r04/c: its workgroups then wait
        // for the arrival ticket instead of returning at once when no winner was deferred)
        const bool tclose = mode == GC_CM_ROUND && !big && (fuse || !d.big_rows) && ticket_close;
        // graphs with big rows: k_commit_big's last workgroup closes the round (GC_CB_CLOSE, round 6;
        // the tickets are counted per dispatch residue, gc_cb_ticket)
        const bool bclose = mode == GC_CM_ROUND && !big && !fuse && d.big_rows && ticket_close && cb_close && d.accs;
        DevCtl* snap = mode == GC_CM_ROUND ? snap_ptr : nullptr;
        kt.begin(mode == GC_CM_INIT ? GC_K_INIT : GC_K_COMMIT);
        gcl_commit(d, L, mode, mode == GC_CM_ROUND && !tail ? -1 : nsweeps, s, big, fuse ? 1 : 0,
                   (tclose || bclose) ? snap : nullptr, tclose ? 1 : (bclose ? 2 : 0));
        kt.end();
        if (mode == GC_CM_ROUND) snap_ptr = nullptr;
        if (tclose || bclose) {
            kt.close();
            proposed = fuse;
            return;
        }
        if (big) {
            kt.begin(GC_K_COMMIT);
            gcl_pull(d, big, s);
            kt.end();
            kt.begin(GC_K_OTHER);
            gcl_front_build(d, L, g->fsum, s);
            kt.end();
        }
        kt.begin(GC_K_OTHER);
        gcl_close(d, L, mode, s, big, fuse ? 1 : 0, snap);
        kt.end();
        kt.close();  // a round's runs end with it
        proposed = fuse;
    }
    void launch_sweeps(int from, int to) {  // sweeps from..to inclusive
        for (int i = from; i <= to; ++i) {
            kt.begin(GC_K_SWEEP);
            gcl_sweep(d, L, i, s);
            kt.end();
        }
    }
    // (round 3's GC_GRAPHS -- each round's launches replayed from a hipGraph -- measured slower
    // in round 4: R-MAT-24 +2.4%, C2 +3.7%, mesh 512^3 +7.3%, profiles/r04/c; removed)
    void enqueue_round(int S) {
        const bool fuse = fuse_now();
        if (!proposed) enqueue_propose();
        kt.begin(GC_K_RESOLVE);
        gcl_resolve(d, L, s);
        kt.end();
        launch_sweeps(1, S);
        launch_commit(GC_CM_ROUND, S, fuse);
    }
    void enqueue_propose() {
        if (resort_hint) {  // device decides; enqueued only while frontiers are within reach of n/64
            kt.begin(GC_K_OTHER);
            gcl_fsort(d, L, g->fsum, s);
            kt.end();
        }
        if (c4_hint) {  // the nibble mirror can only pay in a big round (k_pack_c4 decides)
            kt.begin(GC_K_OTHER);
            gcl_pack_c4(d, s);
            kt.end();
        }
        const bool inl = inline_now();
        kt.begin(GC_K_PROPOSE);
        gcl_propose(d, L, s, resort_hint ? 0 : 1, inl ? 1 : 0);
        kt.end();
        if (need_pblock() && !inl) {  // heavy (deg > heavy_t) or wide (mex >= 64, so deg >= 64) proposers possible
            kt.begin(GC_K_PROPOSE);
            gcl_propose_block(d, L, s);
            kt.end();
        }
    }
    // a batch of rounds followed by an async snapshot of the control block
    // The batch's last k_close writes the snapshot into the pinned slot itself (a copy
    // engine blit of the control block cost ~16 us of stream time per batch; GC_SNAP_COPY=1
    // restores it for A/B measurements).
    const bool snap_copy = getenv("GC_SNAP_COPY") && atoi(getenv("GC_SNAP_COPY")) > 0;
    DevCtl* snap_ptr = nullptr;  // handed to the next round's k_close (or closing commit)
    // GC_TICKET_CLOSE=0: always a separate k_close launch (A/B measurements)
    const bool ticket_close = !(getenv("GC_TICKET_CLOSE") && atoi(getenv("GC_TICKET_CLOSE")) == 0);
    // GC_CB_CLOSE=1: graphs with big rows close the round in k_commit_big's last workgroup instead
    // of a k_close launch (round 6: neutral on R-MAT-24, 142.30 vs 142.26 ms, profiles/r06/u; off,
    // so the per-round trace views keep finding one closing kernel per round)
    const bool cb_close = getenv("GC_CB_CLOSE") && atoi(getenv("GC_CB_CLOSE")) > 0;
    int enqueue_batch(int B, int S, int slot) {
        if (core_pending) {  // between rounds: the colours it reads are a round start
            kt.begin(GC_K_OTHER);
            gcl_core_build(d, s);
            kt.end();
            core_pending = false;
        }
        for (int b = 0; b < B; ++b) {
            if (b == B - 1 && !snap_copy) snap_ptr = g->hsnap_dev + slot;
            enqueue_round(S);
        }
        kt.close();
        if (snap_copy) GC_HIP(hipMemcpyAsync(&g->hsnap[slot], g->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, s));
        GC_HIP(hipEventRecord(g->evsnap[slot], s));
        return GC_OK;
    }
    // sweeps to enqueue per round from the depths seen so far: none while every round
    // was decided by the first sweep (meshes), else twice the last round's depth
    const int sweep_pad = getenv("GC_SWEEP_PAD") ? atoi(getenv("GC_SWEEP_PAD")) : 2;
    bool skip_tail = false;  // set with S = 0 once 16 rounds ran without a second sweep
    int pick_sweeps(const DevCtl& h) {
        skip_tail = h.maxdepth <= 1 && h.round >= 16;
        if (h.maxdepth <= 1 || async_grid > 0) return 0;  // k_sweep_async takes the whole chain
        // the small-list tail runs in k_sweep_tail; with the loop kernel, the full grid only
        // takes the sweeps past its limits
        if (loop_grid > 0) return (int)std::min<long long>(64, h.lasthuge + 1);
        return (int)std::min<long long>(64, h.lastbig + sweep_pad);
    }
    // rounds per batch: small while the frontier is tiny or the colouring is nearly done
    int pick_batch(const DevCtl& h, long long n, int prev) const {
        if (h.U * 64 < n) return 1;
        return std::min(prev * 2, std::max(1, batch_max));
    }
    static bool pick_c4(const DevCtl& h, long long n) { return (long long)h.fcnt[h.cur] * 64 >= n && h.maxcolor < 14; }

    // E1: every component of the uncoloured-induced subgraph gets its
    // argmax-(deg, pos) vertex as a colour-0 seed; committed like a round's winners.
    int e1_reseed() {
        int rc;
        GC_HIP(hipMemsetAsync(&g->ctl->list_cnt, 0, sizeof(ull), s));
        GC_HIP(hipMemsetAsync(&g->ctl->seed_cnt[0], 0, 2 * sizeof(ull), s));
        const int gridn = gc_grid_for_waves(g->n);
        kt.begin(GC_K_RESEED);
        gcl_unc_compact(d, g->ulist, &g->ctl->list_cnt, g->parent, g->best, gridn, s);
        kt.end();
        if ((rc = sync_ctl())) return rc;
        const long long Lc = (long long)g->hctl->list_cnt;
        kt.begin(GC_K_RESEED);
        gcl_cc_hook(d, g->ulist, &g->ctl->list_cnt, g->parent, gc_grid_for_waves(Lc), s);
        kt.end();
        kt.begin(GC_K_RESEED);
        gcl_cc_best(d, g->ulist, &g->ctl->list_cnt, g->parent, g->best, gc_grid_for_waves(Lc, 4096), s);
        kt.end();
        kt.begin(GC_K_RESEED);
        gcl_cc_seeds(d, g->ulist, &g->ctl->list_cnt, g->parent, g->best, g->seeds[0], g->seeds[1],
                     gc_grid_for_waves(Lc, 4096), s);
        kt.end();
        kt.begin(GC_K_RESEED);
        gcl_commit(d, L, GC_CM_RESEED, 0, s);
        kt.end();
        kt.begin(GC_K_RESEED);
        gcl_close(d, L, GC_CM_RESEED, s);
        kt.end();
        return GC_OK;
    }

    // rs != null (gc_color_resume): the state at the start of round rs->round0 comes from the
    // caller's colours and frontier instead of init + seed
    int go(int32_t* colors_out, int32_t* cround_out, const ResumeArgs* rs = nullptr) {
        int rc;
        DevCtl& h = *g->hctl;
        memset(&h, 0, sizeof(DevCtl));
        h.kbound = opt->num_colors;
        h.e1 = opt->e1 ? 1 : 0;
        h.rcap = g->rcap;
        h.maxmex = -1;
        h.nx_maxmex = -1;
        h.hub_start = GC_HUB_NOT_STARTED;
        h.maxcolor = -1;
        h.fail_round = -1;
        h.want_cround = cround_out != nullptr;
        h.pull_off = getenv("GC_NO_PULL") ? 1 : 0;
        h.core_round = -1;
        if (rs) {
            h.round = rs->round0;
            h.rbase = rs->round0;
            h.cur = 0;
            h.fcnt[0] = (ull)rs->nf;
            drained = rs->round0;
        }
        GC_HIP(hipMemcpyAsync(g->ctl, &h, sizeof(DevCtl), hipMemcpyHostToDevice, s));
        GC_HIP(hipMemsetAsync(g->bstat, 0, sizeof(ull) * GC_STAT_SLOTS * 16, s));
        GC_HIP(hipEventRecord(g->ev0, s));
        if (rs) {  // the caller's state (the E1 list and its count serve as the hub pushes' scratch)
            kt.begin(GC_K_INIT);
            gcl_resume(d, L, rs->colors, rs->cround, rs->front, rs->nf, g->ulist, &g->ctl->list_cnt, s);
            kt.end();
            GC_HIP(hipMemsetAsync(&g->ctl->list_cnt, 0, sizeof(ull), s));
        } else {
        // init + seed (coloring.py:74-76)
        kt.begin(GC_K_INIT);
        gcl_init(d, g->seeds[0], gc_grid_for_waves(g->n), s);
        kt.end();
        kt.begin(GC_K_INIT);
        gcl_seed_prep(d, g->seeds[0], g->seeds[1], s);
        kt.end();
        launch_commit(GC_CM_INIT, 0);
        }
        const long long max_rounds = 4ll * g->n + 16;
        // Pipelined: batch k+1 is enqueued before the host waits on batch k's snapshot, so
        // the device never idles on the host.  Any halt drains the stream and is handled on
        // the synchronous path below, then the pipeline restarts.
        int batch = 1, S = 1;
        for (;;) {
            int slot = 0;
            if ((rc = enqueue_batch(batch, S, slot))) return rc;
            for (;;) {
                if ((rc = enqueue_batch(batch, S, slot ^ 1))) return rc;
                GC_HIP(hipEventSynchronize(g->evsnap[slot]));
                const DevCtl& sn = g->hsnap[slot];
                if (sn.halt != GC_RUN || sn.loop_err >= 2) break;
                if (sn.round > max_rounds) { gc_set_error("round limit exceeded"); return GC_EROUNDS; }
                resort_hint = (long long)sn.fcnt[sn.cur] * 256 >= g->n;
                maxc_hint = sn.maxcolor;
                core_check(sn);
                S = pick_sweeps(sn);
                c4_hint = pick_c4(sn, g->n);
                batch = pick_batch(sn, g->n, batch);
                slot ^= 1;
            }
            if ((rc = sync_ctl())) return rc;
            if (h.loop_err >= 2) break;  // reported below
            proposed = h.proposed != 0;
            if (h.round > max_rounds) { gc_set_error("round limit exceeded"); return GC_EROUNDS; }
            int halt = h.halt;
            // a round deeper than the sweeps enqueued: finish its sweeps, then its commit
            while (halt == GC_H_SWEEPS) {
                const int done = (int)h.sweeps_enq;
                if (done > g->n + 64) { gc_set_error("Jones-Plassmann sweeps do not converge"); return GC_EROUNDS; }
                const int more = std::max(4, done);
                if ((rc = clear_halt())) return rc;
                launch_sweeps(done + 1, done + more);
                launch_commit(GC_CM_ROUND, done + more, fuse_now());
                if ((rc = sync_ctl())) return rc;
                halt = h.halt;
            }
            proposed = h.proposed != 0;
            resort_hint = (long long)h.fcnt[h.cur] * 256 >= g->n;
            maxc_hint = h.maxcolor;
            core_check(h);
            S = pick_sweeps(h);
            c4_hint = pick_c4(h, g->n);
            batch = pick_batch(h, g->n, 1);
            if (halt == GC_RUN) continue;
            if (halt == GC_H_DONE || halt == GC_H_FAILED || halt == GC_H_STALLED) break;
            if (halt == GC_H_ROUNDCAP) {
                if ((rc = drain_records()) || (rc = clear_halt())) return rc;
                continue;
            }
            if (halt == GC_H_RESEED) {
                if ((rc = drain_records())) return rc;
                if ((rc = clear_halt()) || (rc = e1_reseed()) || (rc = sync_ctl())) return rc;
                proposed = false;
                if (h.halt == GC_H_DONE) break;
                if (h.halt == GC_H_RESEED || h.halt == GC_H_ROUNDCAP || h.halt == GC_H_STALLED) {
                    // handled by the synchronous path of the next pass (no rounds run first)
                    continue;
                }
                batch = 1;
                continue;
            }
            gc_set_error("unexpected device halt code %d", halt);
            return GC_EHIP;
        }
        if (h.loop_err == GC_LERR_INL) { gc_set_error("k_propose: a hub bitmap does not cover the colours in use (round %lld)", h.round); return GC_EHIP; }
        if (h.loop_err == GC_LERR_LIST) { gc_set_error("a work-list append passed the list's capacity (round %lld)", h.round); return GC_EHIP; }
        if (h.loop_err == 2) { gc_set_error("k_sweep_async: undecided list count out of range"); return GC_EHIP; }
        if (h.loop_err == 4) { gc_set_error("gc_color_resume: a frontier entry is out of range"); return GC_EINVAL; }
        if (h.loop_err == 3) {
            gc_set_error("GC_CHECKS: out-of-range value code %lld (%lld, %lld, %lld) in round %lld", h.dbg[0], h.dbg[1],
                         h.dbg[2], h.dbg[3], h.round);
            return GC_EHIP;
        }
        if (h.loop_err) { gc_set_error("k_sweep_loop: a grid barrier wait gave up"); return GC_EHIP; }
        kt.begin(GC_K_OTHER);
        gcl_finalize(d, gc_grid_for_waves(g->n, 8192), s);
        gcl_stat_reduce(d, s);
        kt.end();
        GC_HIP(hipEventRecord(g->ev1, s));
        if (colors_out) GC_HIP(hipMemcpyAsync(colors_out, g->color, sizeof(int) * g->n, hipMemcpyDeviceToHost, s));
        if (cround_out) GC_HIP(hipMemcpyAsync(cround_out, g->cround, sizeof(int) * g->n, hipMemcpyDeviceToHost, s));
        if ((rc = sync_ctl())) return rc;
        if ((rc = drain_records())) return rc;
        if (core_debug)
            fprintf(stderr, "[gc core] %lld of %zu rounds decided by the core: %lld iterations (max %lld)\n",
                    h.core_handled, recs.size(), h.core_iters_sum, h.core_iters_max);
#ifdef GC_A_PROF
        gcl_aprof_dump(recs.data(), recs.size());
#endif
        GC_HIP(hipGetLastError());
        const int status = h.halt == GC_H_FAILED ? GC_FAILED : (h.halt == GC_H_STALLED ? GC_STALLED : GC_OK);
        if (st) {
            float ms = 0.f;
            GC_HIP(hipEventElapsedTime(&ms, g->ev0, g->ev1));
            st->device_ms = ms;
            st->rounds = (long long)recs.size();
            st->max_color = h.maxcolor;
            st->jp_sweeps = h.sweep_total;
            st->async_aborts = (int64_t)h.async_aborts;
            st->hubs = d.hbits_w ? (int64_t)g->nhub : 0;
            st->core_rounds = (int64_t)h.core_handled;
            st->fail_round = h.halt == GC_H_FAILED ? h.fail_round : -1;
            st->fail_count = h.halt == GC_H_FAILED ? h.fail_count : 0;
            for (const RoundRec& r : recs) st->reseeds += r.seeds;
            for (long long i = 0; i < (long long)recs.size() && i < st->round_cap; ++i) {
                const RoundRec& r = recs[(size_t)i];
                if (st->round_U) st->round_U[i] = r.U;
                if (st->round_F) st->round_F[i] = r.F;
                if (st->round_maxmex) st->round_maxmex[i] = r.maxmex;
                if (st->round_accepted) st->round_accepted[i] = r.accepted;
                if (st->round_seeds) st->round_seeds[i] = r.seeds;
            }
            // SURVEY.md §8d algorithmic bytes per kernel class
            st->k_bytes[GC_K_PROPOSE] = 24.0 * (double)h.nvert[GC_K_PROPOSE] + 8.0 * (double)h.sumdeg[GC_K_PROPOSE];
            st->k_bytes[GC_K_RESOLVE] = 24.0 * (double)h.nvert[GC_K_RESOLVE] + 12.0 * (double)h.sumdeg[GC_K_RESOLVE];
            st->k_bytes[GC_K_COMMIT] = 16.0 * (double)h.nvert[GC_K_COMMIT] + 8.0 * (double)h.sumdeg[GC_K_COMMIT];
            kt.collect();
        }
        return status;
    }
};

}  // namespace

// GC_PREP_TIMING=1: host-side phase times of a colouring's set-up on stderr (each phase ends
// in a stream synchronisation; gc_hubs.hip prints the hub index's own phases)
struct ColourClock {
    bool on = getenv("GC_PREP_TIMING") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(const char* what, hipStream_t s) {
        if (!on) return;
        hipStreamSynchronize(s);
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[gc color] %-14s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
};

static int color_impl(gc_graph* g, const gc_options* opt, int32_t* colors_out, int32_t* cround_out, gc_stats* stats,
                      const ResumeArgs* rs) {
    if (!g || !opt) { gc_set_error("gc_color: null argument"); return GC_EINVAL; }
    if (opt->variant != GC_VARIANT_A && opt->variant != GC_VARIANT_B) {
        gc_set_error("gc_color: unknown variant %d", opt->variant);
        return GC_EINVAL;
    }
    GC_HIP(hipSetDevice(g->device));
    ColourClock cc;
    int rc = gc_alloc_run_state(g);
    if (rc) return rc;
    cc.mark("run state", g->stream);
    auto clear_stats = [&]() {
        if (!stats) return;
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
    };
    clear_stats();
    if (opt->variant == GC_VARIANT_B && (opt->priority != GC_PRIORITY_REF || opt->speculative)) {
        gc_set_error("gc_color: seeded priorities and the speculative mode are variant A only");
        return GC_EINVAL;
    }
    if (rs && (opt->variant != GC_VARIANT_A || opt->priority != GC_PRIORITY_REF || opt->speculative)) {
        gc_set_error("gc_color_resume: variant A with the reference rank only");
        return GC_EINVAL;
    }
    // the rows are partitioned for the rank of this colouring (re-partitioned when it changes)
    if ((rc = gc_set_priority(g, opt->priority, opt->seed))) return rc;
    cc.mark("priority", g->stream);
    if (opt->variant == GC_VARIANT_B) return gc_color_variant_b(g, opt, colors_out, cround_out, stats);
    if (opt->speculative) return gc_color_speculative(g, opt, colors_out, cround_out, stats);
    for (int attempt = 0;; ++attempt) {
    Run run{g, opt, stats, KTimer{g, (unsigned)opt->kernel_timing, stats}, gc_view(g), gc_lists(g), g->stream,
            {}, 0};
    if (attempt) run.inline_pb = false;
    // hubs: forbidden-colour bitmaps for their proposals; the hub JP (hubs rank above every
    // light vertex) only under (deg, pos) -- seeded ranks resolve hubs by row scans
    if ((rc = gc_hubs_prepare(g, run.d))) return rc;
    cc.mark("hubs", g->stream);
    if (opt->priority != GC_PRIORITY_REF) {
        run.d.hub_w = 0;
        run.d.tail_hmax = GC_TAIL_HMAX;
    }
    if (run.d.hub_w == 0 && g->maxdeg > run.d.heavy_t) {
        run.d.heavy_wg = 1;
        if ((rc = gc_alloc_heavy_pending(g))) return rc;
        run.d.hpl = g->hpl;
        run.d.hplc = g->hplc;
    }
    run.init_loop();
    run.init_async();
    {
        const char* f = getenv("GC_FUSE");
        run.fuse_ok = !run.need_pblock() && run.d.hub_w == 0 && !(f && atoi(f) == 0);
    }
    run.d.accs = g->accs;
    GC_HIP(hipMemsetAsync(g->accs, 0, sizeof(ull) * (GC_ACC_SLOTS + GC_TICK_WORDS), g->stream));
    cc.mark("set-up", g->stream);
    rc = run.go(colors_out, cround_out, rs);  // stats->rounds may exceed round_cap: the caller re-asks
    cc.mark("rounds", g->stream);
    // A hub proposed inside k_propose<1> whose bitmap no longer covered the colours in use (the
    // host's margin on the last snapshot's max colour was too small: never seen) is reported by
    // the device as GC_LERR_INL; the colouring is then run again without the inlined proposals
    // (k_propose_block scans such a hub's row) instead of failing.
    if (rc == GC_EHIP && attempt == 0 && run.inline_pb && g->hctl->loop_err == GC_LERR_INL) {
        clear_stats();
        continue;
    }
    return rc;
    }
}

extern "C" int gc_color(gc_graph* g, const gc_options* opt, int32_t* colors_out, int32_t* cround_out,
                        gc_stats* stats) {
    return color_impl(g, opt, colors_out, cround_out, stats, nullptr);
}

extern "C" int gc_color_resume(gc_graph* g, const gc_options* opt, const int32_t* colors_dev, const int32_t* cround_dev,
                               const int32_t* front_dev, int64_t nfront, int64_t round0, int32_t* colors_out,
                               int32_t* cround_out, gc_stats* stats) {
    if (!g || !colors_dev || (nfront > 0 && !front_dev) || nfront < 0 || nfront > g->n || round0 < 0) {
        gc_set_error("gc_color_resume: bad argument");
        return GC_EINVAL;
    }
    // the caller's device buffers may still be being written on another stream (torch's):
    // the library's own stream is non-blocking, so order its first read after them
    GC_HIP(hipSetDevice(g->device));
    if (int rc = gc_order_after_inputs(g->stream)) return rc;
    const ResumeArgs rs{colors_dev, cround_dev, front_dev, (long long)nfront, (long long)round0};
    return color_impl(g, opt, colors_out, cround_out, stats, &rs);
}

extern "C" int gc_validate(gc_graph* g, const int32_t* colors, int64_t* uncolored, int64_t* conflicts) {
    if (!g) { gc_set_error("gc_validate: null graph"); return GC_EINVAL; }
    return gc_validate_range(g, colors, 0, g->n, uncolored, conflicts);
}

extern "C" int gc_validate_range(gc_graph* g, const int32_t* colors, int64_t lo, int64_t hi, int64_t* uncolored,
                                 int64_t* conflicts) {
    if (!g) { gc_set_error("gc_validate: null graph"); return GC_EINVAL; }
    if (lo < 0 || hi > g->n || lo > hi) {
        gc_set_error("gc_validate_range: [%lld, %lld) is not within [0, %lld)", (long long)lo, (long long)hi, g->n);
        return GC_EINVAL;
    }
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
    // the resident colouring (colors == null): its neighbours' colours gathered from the byte
    // mirror c8 (n bytes instead of 4n of random-gather footprint: 67 MB against 268 MB on
    // R-MAT-26; bit-exact, tests/test_gpu_parity.py); GC_VALIDATE_C8=0 gathers the int colours
    const bool c8 = !colors && !(getenv("GC_VALIDATE_C8") && atoi(getenv("GC_VALIDATE_C8")) == 0);
    if ((rc = gc_validate_tiles(g, src, c8 ? g->c8 : nullptr, lo, hi))) return rc;
    GC_HIP(hipMemcpyAsync(g->hctl, g->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, g->stream));
    GC_HIP(hipStreamSynchronize(g->stream));
    if (uncolored) *uncolored = (int64_t)g->hctl->uncolored;
    if (conflicts) *conflicts = (int64_t)g->hctl->conflicts;
    return GC_OK;
}
