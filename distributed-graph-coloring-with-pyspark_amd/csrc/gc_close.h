#pragma once
// gc_close.h -- the end of a round (k_close, or the last workgroup of a closing commit):
// records, the control block's reset for the next round, the start-of-round checks.  Plain
// single-thread code over the control block, __host__ __device__ so that tests/host_close
// checks the batched form (GC_CLOSE_BATCH) against the interleaved one on the CPU.
#include "gc_device.h"

// the current frontier is big (>= n/64): the big-round machinery may run
__host__ __device__ __forceinline__ bool gc_resort_on(const GDev& g, const DevCtl* c) {
    return (long long)c->fcnt[c->cur] * 64 >= (long long)g.n && c->fcnt[c->cur] > 0;
}
__host__ __device__ __forceinline__ bool gc_big_on(const GDev& g, const DevCtl* c) { return gc_resort_on(g, c); }
__host__ __device__ __forceinline__ bool gc_front_on(const GDev& g, const DevCtl* c, int allow_big) {
    return allow_big && !c->halt && gc_big_on(g, c);
}

__host__ __device__ __forceinline__ void gc_record(const GLists& L, DevCtl* c, long long U, long long F,
                                                   long long maxmex, long long acc, long long seeds, long long sweeps) {
    RoundRec* rec = L.rec + (c->round - c->rbase);
    rec->U = U;
    rec->F = F;
    rec->maxmex = maxmex;
    rec->accepted = acc;
    rec->seeds = seeds;
    rec->sweeps = sweeps;
    gc_st(&c->round, c->round + 1);
}

// Start-of-round checks (coloring.py:86-95 plus E1): U == 0 ends the colouring; no
// proposer with uncoloured vertices left either stalls (E1 off: the reference spins
// forever) or asks the host for an E1 re-seed.
__host__ __device__ __forceinline__ void gc_precheck(const GLists& L, DevCtl* c, long long U, long long F) {
    if (U == 0) {
        gc_record(L, c, 0, 0, -1, 0, 0, 0);
        gc_st(&c->halt, (int)GC_H_DONE);
    } else if (F == 0) {
        if (!c->e1) {
            gc_record(L, c, U, 0, -1, 0, 0, 0);
            gc_st(&c->halt, (int)GC_H_STALLED);
        } else {
            gc_st(&c->halt, (int)GC_H_RESEED);
        }
    } else if (c->round - c->rbase + 4 >= c->rcap) {
        gc_st(&c->halt, (int)GC_H_ROUNDCAP);
    }
}

// Run by ONE thread of the last workgroup of a commit, after every other workgroup's
// counter atomics (counters are read back with atomic RMWs, written with agent-scope
// stores; the next kernel reads them after the launch boundary).
// A fused commit (k_commit<1>) made the next round's proposals: their failure count and
// max candidate move from the nx_ slots into place (else the nx_ slots hold 0 / -1).
// pre (gc_close_body): the counters it needs, read by separate lanes in one memory trip
struct GcClosePre {
    ull accepted, nx_failcnt, uncolored, fnext;
    long long nx_maxmex;
};
// GC_CLOSE_INLINE (build knob, default 1 since round 3): the close is inlined into k_commit /
// k_close.  As a call (0, rounds 1-2) it gave both kernels a 176-byte private segment --
// scratch set up for every wave of every launch -- for the one workgroup that closes the
// round; inlined, no round kernel uses scratch (k_commit<0> 59 -> 69 VGPRs).
#ifndef GC_CLOSE_INLINE
#define GC_CLOSE_INLINE 1
#endif
#if GC_CLOSE_INLINE
#define GC_CLOSE_ATTR __attribute__((always_inline)) inline
#else
#define GC_CLOSE_ATTR __attribute__((noinline))
#endif
__host__ __device__ GC_CLOSE_ATTR void gc_close_round(const GLists& L, DevCtl* c, int mode, int fused,
                                                    const GcClosePre& pre) {
    const long long acc = (long long)pre.accepted;
    long long U = c->U;
    int cur = c->cur;
    if (mode == GC_CM_ROUND) {
        const long long F = (long long)c->fcnt[cur];
        const long long sw = c->sweeps;
        gc_st(&c->sweep_total, c->sweep_total + (sw > 0 ? sw - 1 : 0));
        if (sw > c->maxdepth) gc_st(&c->maxdepth, sw);
        gc_st(&c->lastdepth, sw);
        gc_st(&c->lastbig, c->bigsweeps);
        gc_st(&c->bigsweeps, 0ll);
        gc_st(&c->lasthuge, c->hugesweeps);
        gc_st(&c->hugesweeps, 0ll);
        gc_record(L, c, U, F, c->maxmex, acc, 0, sw);
        U -= acc;
        gc_st(&c->fcnt[cur], 0ull);  // becomes the next round's output slot
        cur ^= 1;
        gc_st(&c->cur, cur);
    } else if (mode == GC_CM_INIT) {
        U = (long long)pre.uncolored - (c->seedkey ? 1 : 0);
    } else {  // GC_CM_RESEED: the E1 round record (no proposers, `acc` seeds planted)
        gc_record(L, c, U, 0, -1, 0, acc, 0);
        U -= acc;
    }
    gc_st(&c->U, U);
    gc_st(&c->heavy_cnt, 0ull);
    gc_st(&c->wide_cnt, 0ull);
    gc_st(&c->failcnt, pre.nx_failcnt);
    gc_st(&c->accepted, 0ull);
    gc_st(&c->maxmex, pre.nx_maxmex);
    gc_st(&c->nx_failcnt, 0ull);
    gc_st(&c->nx_maxmex, -1ll);
    gc_st(&c->proposed, mode == GC_CM_ROUND && fused ? 1 : 0);
    gc_st(&c->sweeps, 0ll);
    gc_st(&c->hub_start, GC_HUB_NOT_STARTED);
    gc_st(&c->loop_last, 0ll);
    for (int k = 0; k < 3; ++k) {
        gc_st(&c->und_cnt[k], 0ull);
        gc_st(&c->undh_cnt[k], 0ull);
    }
    gc_st(&c->seed_cnt[0], 0ull);
    gc_st(&c->bigw_cnt, 0ull);
    gc_st(&c->use_c4, 0);  // k_pack_c4 (when the host enqueues it) turns it on for its round
    gc_st(&c->seed_cnt[1], 0ull);
    gc_precheck(L, c, U, (long long)pre.fnext);
}

// the close as rounds 1-3 run it (gc_close_body's closing thread): the next list's order, then
// gc_close_round
__host__ __device__ __forceinline__ void gc_close_interleaved(const GDev& g, const GLists& L, DevCtl* c, int mode,
                                                              int allow_big, int fused, const GcClosePre& pre) {
    c->sorted = mode == GC_CM_ROUND && gc_front_on(g, c, allow_big);  // next list built in order
    gc_close_round(L, c, mode, fused, pre);
}

// GC_CLOSE_BATCH (build knob, default 1 since round 3; 0 = the interleaved form, variant
// close_interleaved of tools/build_staged.sh): the close as ONE batch of loads and then the
// stores.  gc_close_round interleaves them (each "store one field, then read
// the next" waits for the store: a wave's loads and stores retire through one counter), so
// the one thread that closes a round walks ~15 dependent L2 round trips -- k_close averaged
// 8.2 us for one wave in round 2 (profiles/latest/rmat24/kernel_stats.csv), on the critical
// path of every round (k_close, or the last workgroup of a ticket-closing commit).  Same
// values, same records, same halts: every field is read before the close writes it, except
// `round`, which is carried in a register across the records it advances -- checked on the
// CPU against the interleaved form over random control blocks (tests/test_host_close.py).
#ifndef GC_CLOSE_BATCH
#define GC_CLOSE_BATCH 1
#endif
struct GcCloseCtl {  // the control words the close reads, as they were when it started
    int halt, cur, e1;
    ull f0, f1, seedkey;
    long long U, sw, swt, maxd, bigs, huges, maxmex, round, rbase, rcap;
};
__host__ __device__ __forceinline__ GcCloseCtl gc_close_load(const DevCtl* c) {
    GcCloseCtl k;
    k.halt = c->halt;
    k.cur = c->cur;
    k.e1 = c->e1;
    k.f0 = c->fcnt[0];
    k.f1 = c->fcnt[1];
    k.seedkey = c->seedkey;
    k.U = c->U;
    k.sw = c->sweeps;
    k.swt = c->sweep_total;
    k.maxd = c->maxdepth;
    k.bigs = c->bigsweeps;
    k.huges = c->hugesweeps;
    k.maxmex = c->maxmex;
    k.round = c->round;
    k.rbase = c->rbase;
    k.rcap = c->rcap;
    return k;
}
// gc_close_body's `sorted` + gc_close_round + gc_precheck from the loaded words
__host__ __device__ __forceinline__ void gc_close_batched(const GDev& g, const GLists& L, DevCtl* c, int mode,
                                                          int allow_big, int fused, const GcClosePre& pre,
                                                          const GcCloseCtl& k) {
    const long long acc = (long long)pre.accepted;
    const ull fcur = k.cur ? k.f1 : k.f0;
    long long U = k.U, round = k.round;
    int cur = k.cur;
    auto record = [&](long long u, long long f, long long mm, long long a, long long sd, long long sw) {
        RoundRec* rec = L.rec + (round - k.rbase);
        rec->U = u;
        rec->F = f;
        rec->maxmex = mm;
        rec->accepted = a;
        rec->seeds = sd;
        rec->sweeps = sw;
        ++round;
    };
    // next list built in order (gc_front_on on the round's own frontier)
    c->sorted = mode == GC_CM_ROUND && allow_big && !k.halt && (long long)fcur * 64 >= (long long)g.n && fcur > 0;
    if (mode == GC_CM_ROUND) {
        gc_st(&c->sweep_total, k.swt + (k.sw > 0 ? k.sw - 1 : 0));
        if (k.sw > k.maxd) gc_st(&c->maxdepth, k.sw);
        gc_st(&c->lastdepth, k.sw);
        gc_st(&c->lastbig, k.bigs);
        gc_st(&c->bigsweeps, 0ll);
        gc_st(&c->lasthuge, k.huges);
        gc_st(&c->hugesweeps, 0ll);
        record(U, (long long)fcur, k.maxmex, acc, 0, k.sw);
        U -= acc;
        gc_st(&c->fcnt[cur], 0ull);  // becomes the next round's output slot
        cur ^= 1;
        gc_st(&c->cur, cur);
    } else if (mode == GC_CM_INIT) {
        U = (long long)pre.uncolored - (k.seedkey ? 1 : 0);
    } else {  // GC_CM_RESEED
        record(U, 0, -1, 0, acc, 0);
        U -= acc;
    }
    gc_st(&c->U, U);
    gc_st(&c->heavy_cnt, 0ull);
    gc_st(&c->wide_cnt, 0ull);
    gc_st(&c->failcnt, pre.nx_failcnt);
    gc_st(&c->accepted, 0ull);
    gc_st(&c->maxmex, pre.nx_maxmex);
    gc_st(&c->nx_failcnt, 0ull);
    gc_st(&c->nx_maxmex, -1ll);
    gc_st(&c->proposed, mode == GC_CM_ROUND && fused ? 1 : 0);
    gc_st(&c->sweeps, 0ll);
    gc_st(&c->hub_start, GC_HUB_NOT_STARTED);
    gc_st(&c->loop_last, 0ll);
    for (int j = 0; j < 3; ++j) {
        gc_st(&c->und_cnt[j], 0ull);
        gc_st(&c->undh_cnt[j], 0ull);
    }
    gc_st(&c->seed_cnt[0], 0ull);
    gc_st(&c->bigw_cnt, 0ull);
    gc_st(&c->use_c4, 0);
    gc_st(&c->seed_cnt[1], 0ull);
    // gc_precheck, with the round counter advanced by the records above
    const long long F = (long long)pre.fnext;
    int halt = GC_RUN;
    if (U == 0) {
        record(0, 0, -1, 0, 0, 0);
        halt = GC_H_DONE;
    } else if (F == 0) {
        if (!k.e1) {
            record(U, 0, -1, 0, 0, 0);
            halt = GC_H_STALLED;
        } else {
            halt = GC_H_RESEED;
        }
    } else if (round - k.rbase + 4 >= k.rcap) {
        halt = GC_H_ROUNDCAP;
    }
    if (round != k.round) gc_st(&c->round, round);
    if (halt != GC_RUN) gc_st(&c->halt, halt);
}
