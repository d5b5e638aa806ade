// gc_launch.h -- kernel argument blocks and the host-side launch wrappers.
#pragma once
#include <hip/hip_runtime.h>
#include "gc_internal.h"

// Graph + run state, passed by value to every kernel.
// Host-side count of the round kernels this thread has launched (every launch in
// gc_kernels.hip, gc_variant_b.hip and gc_priority.hip goes through GC_LAUNCH): KTimer
// attributes the launches between two class switches to the class, so a bracket that
// enqueues two kernels (gcl_commit: k_commit + k_commit_big) counts two.
extern thread_local long long gc_tl_launches;
#define GC_LAUNCH(...)                    \
    do {                                  \
        ++gc_tl_launches;                 \
        hipLaunchKernelGGL(__VA_ARGS__);  \
    } while (0)

struct GDev {
    int n;
    long long nnz;
    long long list_cap;  // entries a staged append may place in a work list (n; GC_TEST_LIST_CAP lowers it in tests)
    const long long* rp;
    const int* col;
    const int* deg;
    const int* nlow;  // lower-rank neighbours listed first in each row
    const long long* trp;  // in-neighbour CSR (== rp/col when symmetric)
    const int* tcol;
    int* color;
    int* cround;
    int* cand;
    unsigned char* c8;
    unsigned* c4;
    unsigned char* k8;
    unsigned int* inF;
    unsigned char* mark;  // big rounds: in-neighbours of the winners (0/1), merged into inF
    DevCtl* ctl;
    int* lcur;            // undecided light vertex: low-row entries a later JP sweep may skip
    ull* bstat;           // GC_STAT_SLOTS x 16 stats slots (gc_stat_add)
    ull* accs;            // GC_ACC_SLOTS winner-count slots (single-GPU engine), else null
    int big_rows;         // some in-row (+ hub row) may exceed bigrow: k_commit_big is needed
    int bigrow;           // heavy winners with longer in-rows (+ hub rows) go to k_commit_big (GC_BIGROW)
    int claim_direct;     // fused commit: claim with one atomic, no check-load first (GC_CLAIM_DIRECT)
    // Shards with replicated hubs (gc_shard.hip): every rank runs the hub JP of every hub, so
    // hubs never travel as deltas, and a rank claims the hubs its winners touched (hseen)
    int hub_repl;
    long long own_lo, own_hi;  // the rank's vertex range (hub_repl: failures counted by owners only)
    int* hseen;               // hub x has a coloured listed neighbour (set by gc_hub_mark), or null
    long long nhub_repl;      //   the number of hubs
    int* hpl;             // hubs-off heavy JP (gc_jp_sweep): heavy v's pending entries at hpl[rp[v] ..], or null
    int* hplc;            //   and their count (written by each sweep of v)
    // Hubs (variant A on one GPU; see gc_hubs.hip).  deg > heavy_t takes the
    // workgroup-per-vertex path; with hubs on (hub_w > 0) every such vertex is a hub that
    // keeps its forbidden colours as a bitmap and its per-round conflict candidates as a
    // list, both pushed to it, instead of re-reading its whole row every round / sweep.
    int heavy_t;
    int hub_w;                // words per hub bitmap (0 = hubs off); > 0 also turns on the hub JP
    int hbits_w;              // words per hub forbidden-colour bitmap for the proposals and the
                              //   commits' pushes (0 = none): == hub_w, or alone (seeded ranks,
                              //   speculative rounds, variant B, whose resolution has no hub JP)
    int tail_hmax;            // heavy entries the one-workgroup tail sweeps may take (GC_TAIL_HMAX[_HUB])
    int b_resident;           // variant B: the asynchronous fold's resident form on (b_async_resident)
    int a_watch;              // variant A's asynchronous JP: held lights between full passes every a_watch-th (0 off)
    int b_watch;              // variant B's asynchronous fold: a full admission rescan every b_watch-th pass, a
                              //   window of b_awin pending entries from the cursor between them (0 off)
    int b_awin;
    int b_refskip;            // variant B's asynchronous fold: a refused admission reads no more entries
    int tail_lmax;            // light entries the tail sweeps may take (GC_TAIL_MAX; env GC_TAIL_LMAX)
    int tail_nw;              // waves of the tail's workgroup: 4, 8 or 16 (env GC_TAIL_WAVES)
    int heavy_wg;             // heavy vertices are resolved a workgroup each (no hub JP, some deg > heavy_t):
                              //   the JP sweeps run on the larger grids (GC_GRID_RH / GC_GRID_SH)
    long long hub_long;       // hub-start sweep: hubs whose hlow row exceeds this are first-read by the whole grid
    const long long* hch_rp;  // static GC_HCH-entry chunks of the hlow rows (hub x: [hch_rp[x], hch_rp[x+1]))
    const int* hch_own;       //   chunk -> hub
    int* hkcnt;               //   kept-row entries written by the grid this round
    long long nhch;
    long long hch_mul;        //   coprime to nhch, ~0.618 nhch: chunk scan order (a long row's chunks spread out)
    int hprep;                // long-row first pass on (GC_HUB_PREP)
    int hub_scan;             // hub JP by a resumable scan of the rank-sorted row (GC_HUB_SCAN, default on)
    unsigned* hk;             // hub x: gc_hk(candidate, state) of hub_v[x], or GC_HK_COLOURED; the hlow rows and
                              //   pending lists hold hub indices, so hub JP gathers this L2-resident mirror
    const int* hid;           // hub index of v, -1 if v is no hub
    const int* hub_v;         // vertex of hub index x
    const long long* hin_rp;  // for every u: the hubs (indices) whose rows list u
    const int* hin_col;
    unsigned* hbits;          // hub x: bit c set <=> a listed neighbour is coloured c (c < 32*hub_w)
    long long hb_stride;      //   hubs of the bitmap array: word t of hub x is hbits[t * hb_stride + x]
                              //   (word-major, GC_HB_WMAJOR; gc_hbw)
    unsigned* hkill;          // hub x, this round: a lower-rank light neighbour it lists won its candidate
    const long long* hlow_rp; // hub x: the lower-rank HUBS its row lists (vertex ids)
    const int* hlow_col;
    int* hcur;                // hub x, this round: 1 once its row was read (gc_hub_jp)
    int* hrow;                // hub x: which copy holds its live row (0 = hlow_col)
    int* hlen;                //   and its length (copies 1, 2)
    int* hlowb[3];            // hlow_col and two working copies (hlow's offsets)
    int* hpc;                 //   undecided same-candidate entries kept in hpend (count << 1 | half)
    int* hpend[2];            //   ping-pong halves, hlow's offsets
    int* hcore;               // hub core (gc_core.hip): hub x -> core index (-1: coloured when the core was built)
    int* core_hub;            //   core index -> hub index
    unsigned* core_bits;      //   core index i -> bitset over core indices: the higher-rank core hubs listing hub i
    ull* core_wcnt;           //   build scratch: uncoloured hubs per workgroup range
    int core_cap;             //   core hubs at most (GC_CORE_MAX, GC_HUB_CORE_CAP lowers it); 0 = no core
    long long nhub_core;      //   hubs of the graph (the build's range)
    int core_iters;           //   winners one class may need in k_hub_core (GC_HUB_CORE_ITERS)
};

// Work lists of the round pipeline (counts live in DevCtl).
struct GLists {
    int* F[2];
    int* heavy;
    int* wide;
    int* undL[3];
    int* undH[3];
    int* seeds[2];
    int* bigw;  // winners with long in-rows (k_commit_big)
    RoundRec* rec;
    long long* delta;  // sharded engine: this phase's outgoing (vertex, value) deltas; else null
};

void gcl_init(const GDev& g, int* seed_light, int grid, hipStream_t s);
void gcl_seed_prep(const GDev& g, int* sl, int* sh, hipStream_t s);
int gcl_fsort_blocks(long long n);
void gcl_fsort(const GDev& g, const GLists& L, unsigned* bsum, hipStream_t s);
void gcl_pack_c4(const GDev& g, hipStream_t s);
void gcl_stat_reduce(const GDev& g, hipStream_t s);
// small: the last frontier was < n/256; inl: heavy and wide proposers here (no k_propose_block)
void gcl_propose(const GDev& g, const GLists& L, hipStream_t s, int small = 0, int inl = 0);
void gcl_propose_block(const GDev& g, const GLists& L, hipStream_t s);
void gcl_resolve(const GDev& g, const GLists& L, hipStream_t s);
void gcl_sweep(const GDev& g, const GLists& L, int i, hipStream_t s);
void gcl_sweep_tail(const GDev& g, const GLists& L, int S, hipStream_t s);  // one-workgroup tail sweeps
void gcl_sweep_loop(const GDev& g, const GLists& L, int S, int grid, hipStream_t s);  // resident-grid sweep chain
// asynchronous JP after sweep S on a resident grid (budget in wall-clock ticks; par alternates per launch)
void gcl_sweep_async(const GDev& g, const GLists& L, int S, int par, long long budget, int grid, hipStream_t s,
                     int lds_lights = 0);
int gcl_sweep_async_blocks_per_cu();
// Workgroups of `block` threads of kernel `fn` that are RESIDENT on a CU at once: the
// runtime's occupancy answer, bounded by what the kernel's own VGPR count and static LDS allow
// (512 VGPRs per SIMD lane in granules of 8, at most 8 waves per SIMD, 160 KB of LDS per CU).
// The runtime answered 8 for k_b_async, whose 66 VGPRs allow 7 waves per SIMD (the compiler's
// resource-usage remark says the same): a grid sized from the runtime's answer had an eighth of
// its workgroups wait for a CU while the resident ones spun on their slices (round 4's
// 8-workgroups-per-CU cliff, R-MAT-24 variant B 365 ms -> 2.0 s).  Persistent and
// asynchronous kernels size their grids from this.
int gc_resident_blocks_per_cu(const void* fn, int block);
// the same, measured on the device: the kernel launched in its residency-probe mode
// (gc_residency_probe), once per device, capped by the runtime's answer
struct gc_graph_ctl_view {
    const GDev* g;
    hipStream_t s;
};
int gc_measure_resident(const void* key, gc_graph_ctl_view v, int query, void (*launch)(const GDev&, int, hipStream_t));
int gcl_sweep_async_resident(const GDev& g, hipStream_t s);
int gcl_b_async_resident(const GDev& g, hipStream_t s);
void gcl_pull(const GDev& g, int allow_big, hipStream_t s);  // pull half of a big round
void gcl_front_build(const GDev& g, const GLists& L, unsigned* bsum, hipStream_t s);  // next list of a big round
// tclose: the commit's last workgroup also closes the round (no k_close; ROUND mode only,
// never with allow_big or when k_commit_big follows); snap: its snapshot slot, or null.
void gcl_commit(const GDev& g, const GLists& L, int mode, int nsweeps, hipStream_t s, int allow_big = 0,
                int fused = 0, DevCtl* snap = nullptr, int tclose = 0);
void gcl_close(const GDev& g, const GLists& L, int mode, hipStream_t s, int allow_big = 0, int fused = 0,
               DevCtl* snap = nullptr);
void gcl_hub_push_big(const GDev& g, const int* big, const ull* cnt, hipStream_t s);  // see gc_hub_push_wave
void gcl_delta_cand(const GDev& g, const GLists& L, hipStream_t s);
void gcl_apply(const GDev& g, int kind, const long long* recv, long long count, long long lo, long long hi, int round,
               int* rwin, hipStream_t s, long long hdr_stride = 0);
void gcl_shard_clear_halt(const GDev& g, int code, hipStream_t s);  // halt := GC_RUN if it is `code`
// big: winners whose hub lists are left to gcl_hub_push_big (counter DevCtl.list_cnt)
void gcl_shard_scan_commit(const GDev& g, const GLists& L, long long lo, long long hi, int* big, hipStream_t s);
void gcl_shard_list_commit(const GDev& g, const GLists& L, const int* rwin, int* big, hipStream_t s);
void gcl_shard_reset(const GDev& g, long long round, hipStream_t s);
void gcl_shard_pack(const GDev& g, int kind, int slot, const long long* delta, long long* send, long long cap,
                    hipStream_t s);
void gcl_shard_flip(const GDev& g, hipStream_t s);
// replicated hubs: the uncoloured hubs a winner touched join the frontier (slot_next: the
// next round's list, else the current one)
void gcl_shard_hub_claim(const GDev& g, const GLists& L, int slot_next, hipStream_t s);
// replicated hubs after a slice seam: the other ranks' light winners flag their hubs
void gcl_shard_hub_flags(const GDev& g, long long lo, long long hi, hipStream_t s);
void gcl_finalize(const GDev& g, int grid, hipStream_t s);
// hub core (gc_core.hip): build attempt (indices + bitsets; does nothing past core_cap uncoloured
// hubs) and the per-round decision of the hubs (before gcl_sweep_async, same S and parity)
void gcl_core_build(const GDev& g, hipStream_t s);
void gcl_hub_core(const GDev& g, const GLists& L, int S, int par, hipStream_t s);
#ifdef GC_A_PROF
void gcl_aprof_dump(const RoundRec* recs, size_t nrec);
void gcl_cprof_dump(FILE* f, size_t nrec);  // gc_core.hip
#endif
void gcl_snap(DevCtl* ctl, DevCtl* snap, hipStream_t s);
// gc_color_resume: the round-start state from colours + frontier (big: scratch list + its count)
void gcl_resume(const GDev& g, const GLists& L, const int* colors, const int* cround, const int* front, long long nf,
                int* big, ull* big_cnt, hipStream_t s);
// a shard's own frontier (its F[cur] without the other ranks' replicated hubs) -> out
void gcl_shard_own_front(const GDev& g, const GLists& L, long long lo, long long hi, int* out, ull* out_cnt,
                         hipStream_t s);
void gcl_unc_compact(const GDev& g, int* list, ull* cnt, int* parent, ull* best, int grid, hipStream_t s);
void gcl_cc_hook(const GDev& g, const int* list, const ull* cnt, int* parent, int grid, hipStream_t s);
void gcl_cc_best(const GDev& g, const int* list, const ull* cnt, int* parent, ull* best, int grid, hipStream_t s);
void gcl_cc_seeds(const GDev& g, const int* list, const ull* cnt, int* parent, const ull* best, int* sl, int* sh,
                  int grid, hipStream_t s);
void gcl_degrees(const long long* rp, int n, long long nnz, int* deg, unsigned char* kb, ull* maxdeg, ull* bad, int grid,
                 hipStream_t s);
