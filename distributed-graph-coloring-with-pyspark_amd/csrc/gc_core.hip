// gc_core.hip -- the hub core: the small rounds' hub JP decided in ONE workgroup (variant A,
// reference rank, one GPU).
//
// Where the small rounds' time went (round 6, -DGC_A_PROF, profiles/r06/a): after the first
// rounds every light proposer decides in the round's first JP sweep (k_resolve), so
// k_sweep_async spends a small round on the hub JP alone -- R-MAT-24's 464 rounds of 1k-16k
// frontier vertices: ~1,900 hub proposers, 11-12 dependent passes, 531k hub-row entries
// scanned, 41 us median; only ~8 hubs win a round.  The uncoloured hubs by then are R-MAT's
// dense core (~80% of the possible hub-hub entries), and an OUT hub's resumable scan walks
// ~280 rank-sorted entries of other candidates before it meets its class's winner.
//
// The core: once the uncoloured hubs fit GC_CORE_MAX (8192), k_core_* index them in rank order
// and store, for every core hub i, the bitset of the higher-rank core hubs whose rows list i
// (from their hlow rows, the coloured prefix skipped: one pass, built once per colouring).  Every
// later hub proposer is a core hub (the uncoloured hubs only shrink).  A round's hub JP is then
// coloring.py:56-70's rule restated for the hubs -- every light ranks below every hub, and the
// lights' winners have already flagged the hubs they kill (hkill):
//   per candidate class, in rank order: a member is IN iff no IN member of its class is listed
//   by it (bit of the member in that winner's bitset);
// which is the lexicographically first maximal independent set the JP sweeps compute.  k_hub_core
// does it in one workgroup, in windows of the 64 lowest-rank undecided proposers (below).  A round
// it cannot take (lights still undecided, more proposers than GC_CORE_MAX, a candidate past
// 65535) is left untouched and k_sweep_async decides it; otherwise it marks the round
// (DevCtl.core_round) and k_sweep_async returns at once.
#include "gc_device.h"
#include "gc_engine.h"

#ifndef GC_CORE_MAX
#define GC_CORE_MAX 8192  // core hubs (and a round's hub proposers) at most: k_hub_core's LDS
#endif
#define GC_CORE_BLOCK 1024
#define GC_CORE_BUILD_GRID 256
static_assert(GC_CORE_MAX % GC_CORE_BLOCK == 0, "k_hub_core holds GC_CORE_MAX / 1024 proposers per thread");

// ------------------------------------------------------------------------------------
// build: uncoloured hubs counted per workgroup range (hub order = rank order)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void core_range(long long nh, long long& a, long long& b) {
    a = nh * blockIdx.x / gridDim.x;
    b = nh * (blockIdx.x + 1) / gridDim.x;
}

__global__ void __launch_bounds__(GC_BLOCK) k_core_count(GDev g, long long nhub) {
    DevCtl* c = g.ctl;
    __shared__ ull scratch[GC_WAVES_PER_BLOCK];
    long long a, b;
    core_range(nhub, a, b);
    ull cnt = 0;
    for (long long x = a + threadIdx.x; x < b; x += blockDim.x) cnt += g.c8[g.hub_v[x]] == GC_C8_NONE ? 1ull : 0ull;
    cnt = gc_wave_sum(cnt);
    const int w = threadIdx.x / GC_WAVE;
    if (gc_lane() == 0) scratch[w] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        ull t = 0;
        for (int i = 0; i < GC_WAVES_PER_BLOCK; ++i) t += scratch[i];
        g.core_wcnt[blockIdx.x] = t;
        if (t) atomicAdd(&c->core_cnt, t);
    }
}

// core indices in hub (= rank) order: hcore[x] for every hub, core_hub[i] for the core
__global__ void __launch_bounds__(GC_BLOCK) k_core_assign(GDev g, long long nhub) {
    DevCtl* c = g.ctl;
    const ull total = c->core_cnt;
    if (total > (ull)g.core_cap || total == 0) {
        if (blockIdx.x == 0 && threadIdx.x == 0) c->core_state = GC_CORE_FAILED;
        return;
    }
    __shared__ ull s_w[GC_WAVES_PER_BLOCK];
    __shared__ int s_c[GC_WAVES_PER_BLOCK];
    const int w = threadIdx.x / GC_WAVE;
    // this range's first core index: the counts of the ranges before it
    ull pre = (threadIdx.x < blockIdx.x) ? g.core_wcnt[threadIdx.x] : 0ull;
    for (unsigned k = threadIdx.x + blockDim.x; k < blockIdx.x; k += blockDim.x) pre += g.core_wcnt[k];
    pre = gc_wave_sum(pre);
    if (gc_lane() == 0) s_w[w] = pre;
    __syncthreads();
    long long base = 0;
    for (int i = 0; i < GC_WAVES_PER_BLOCK; ++i) base += (long long)s_w[i];
    __syncthreads();
    long long a, b;
    core_range(nhub, a, b);
    for (long long x0 = a; x0 < b; x0 += blockDim.x) {
        const long long x = x0 + threadIdx.x;
        const bool unc = x < b && g.c8[g.hub_v[x]] == GC_C8_NONE;
        const ull m = __ballot(unc);
        if (gc_lane() == 0) s_c[w] = __popcll(m);
        __syncthreads();
        long long off = base;
        for (int i = 0; i < w; ++i) off += s_c[i];
        long long step = 0;
        for (int i = 0; i < GC_WAVES_PER_BLOCK; ++i) step += s_c[i];
        if (x < b) {
            const int idx = unc ? (int)(off + __popcll(m & gc_lanemask_lt())) : -1;
            g.hcore[x] = idx;
            if (unc) g.core_hub[idx] = (int)x;
        }
        base += step;
        __syncthreads();
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        c->core_n = (int)total;
        c->core_state = GC_CORE_READY;
    }
}

__global__ void __launch_bounds__(GC_BLOCK) k_core_zero(GDev g) {
    DevCtl* c = g.ctl;
    if (c->core_state != GC_CORE_READY) return;
    const long long nc = c->core_n, W = (nc + 31) / 32;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nc * W; i += (long long)gridDim.x * blockDim.x)
        g.core_bits[i] = 0u;
}

// a wave per core hub j: every core hub i its row lists below it gets bit j in its bitset
// (entries before hlen[x] are coloured: no core hub there)
__global__ void __launch_bounds__(GC_BLOCK) k_core_bits(GDev g) {
    DevCtl* c = g.ctl;
    if (c->core_state != GC_CORE_READY) return;
    const int nc = c->core_n;
    const long long W = (nc + 31) / 32;
    const int lane = gc_lane();
    for (long long j = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + threadIdx.x / GC_WAVE; j < nc;
         j += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
        const int x = g.core_hub[j];
        const long long e0 = g.hlow_rp[x] + g.hlen[x], e1 = g.hlow_rp[x + 1];
        const unsigned bit = 1u << (j & 31);
        for (long long e = e0 + lane; e < e1; e += GC_WAVE) {
            const int ci = g.hcore[g.hlow_col[e]];
            if (ci >= 0) atomicOr(&g.core_bits[(long long)ci * W + (j >> 5)], bit);
        }
    }
}

// ------------------------------------------------------------------------------------
// the round's hub JP in one workgroup (after k_resolve: slot S = 0 undecided lists)
// ------------------------------------------------------------------------------------
#ifdef GC_A_PROF
// (diagnostic build: per round, the core's proposers, killed ones, classes, largest class,
// iterations and winners; dumped with the asynchronous JP's records, GC_A_PROF_OUT)
#define GC_C_PROF_ROUNDS 4096
__device__ ull gc_cprof[GC_C_PROF_ROUNDS][8];
__device__ ull gc_tstep[GC_C_PROF_ROUNDS][8];
void gcl_cprof_dump(FILE* f, size_t nrec) {
    static ull hb[GC_C_PROF_ROUNDS][8];
    if (hipMemcpyFromSymbol(hb, HIP_SYMBOL(gc_cprof), sizeof(hb)) != hipSuccess) return;
    static ull ts[GC_C_PROF_ROUNDS][8];
    if (hipMemcpyFromSymbol(ts, HIP_SYMBOL(gc_tstep), sizeof(ts)) != hipSuccess) return;
    fprintf(f, "# core: r proposers setup_ticks windows_ticks words_per_row windows winners handled step1 step2 step3 step4 (10 ns ticks)\n");
    for (size_t i = 0; i < nrec && i < GC_C_PROF_ROUNDS; ++i)
        if (hb[i][0])
            fprintf(f, "C %zu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu\n", i, hb[i][0], hb[i][1], hb[i][2],
                    hb[i][3], hb[i][4], hb[i][5], hb[i][6], ts[i][1], ts[i][2], ts[i][3], ts[i][4], ts[i][5], ts[i][6]);
    static ull z[GC_C_PROF_ROUNDS][8];
    (void)hipMemcpyToSymbol(HIP_SYMBOL(gc_cprof), z, sizeof(z));
}
#endif

// The round's hub JP in windows of the 64 lowest-rank undecided proposers (every class at once;
// R-MAT's small rounds have ONE class of ~2,000 hub proposers with ~8 winners, profiles/r06/c).
// Thread t holds proposers t + k * 1024 (k < 8) in registers; the undecided ones are bits of an
// LDS bitmap over core indices (= rank order).  A window:
//   1. wave 0 lists the bitmap's first 64 set bits (the lowest-rank undecided proposers);
//   2. the workgroup loads their 64 bitsets into LDS (one coalesced trip);
//   3. wave 0 decides the window in rank order from those bits alone: member j is IN iff no
//      earlier IN member of its class is listed by it (bit of j in that member's bitset) --
//      every lower-rank member of its class is decided: in an earlier window, or earlier here;
//   4. every other undecided proposer whose row lists one of the window's winners of its class
//      is OUT (LDS bit tests); the decided ones leave the bitmap.
// So each window decides at least 64 proposers: at most 128 windows, one global trip each.
#define CORE_WIN 64
__global__ void __launch_bounds__(GC_CORE_BLOCK) k_hub_core(GDev g, GLists L, int S, int par) {
    DevCtl* c = g.ctl;
    if (c->halt || c->core_state != GC_CORE_READY) return;
    const long long j = S;
    const int in = (int)(j % 3), z = (int)((j + 2) % 3);
    const long long cl = (long long)c->und_cnt[in];
    const long long ch = (long long)c->heavy_cnt;
    const bool started = c->hub_start <= j;
    if (cl != 0 || ch <= 0 || ch > GC_CORE_MAX || started) return;  // k_sweep_async takes the round
#ifdef GC_A_PROF
    const ull tp0 = wall_clock64();
#endif
    constexpr int WMAX = GC_CORE_MAX / 32;
    __shared__ unsigned s_und[WMAX];                 // undecided proposers, by core index
    __shared__ unsigned short s_cc[GC_CORE_MAX];     // candidate of core index (valid while undecided)
    __shared__ unsigned char s_wpos[GC_CORE_MAX];    // window slot of core index (valid in its window)
    __shared__ unsigned s_rows[CORE_WIN][WMAX + 1];  // the window's bitsets (+1: lane i reading row i
                                                     // at one column hits bank i, not one bank 64 times)
    __shared__ int s_win[CORE_WIN];
    __shared__ int s_bad, s_wt[WMAX / GC_WAVE];
    __shared__ ull s_inmask, s_P[CORE_WIN];
    const int t = threadIdx.x, lane = gc_lane();
    if (t == 0) s_bad = 0;
    for (int b = t; b < WMAX; b += GC_CORE_BLOCK) s_und[b] = 0u;
    __syncthreads();
    const int n = (int)ch, cn = c->core_n;
    const int Wc = (cn + 31) / 32;
    constexpr int U = GC_CORE_MAX / GC_CORE_BLOCK;
    int v[U], x[U], ci[U], cand[U];
    unsigned st[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = t + k * GC_CORE_BLOCK < n ? L.heavy[t + k * GC_CORE_BLOCK] : -1;
    unsigned kv[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
        x[k] = v[k] >= 0 ? g.hid[v[k]] : -1;
        kv[k] = v[k] >= 0 ? (unsigned)g.k8[v[k]] : 0u;
    }
    bool bad = false;
#pragma unroll
    for (int k = 0; k < U; ++k) {
        st[k] = GC_JP_OUT;
        ci[k] = 0;
        cand[k] = 0;
        if (v[k] < 0) continue;
        const unsigned c6 = gc_k8_cand(kv[k]);
        cand[k] = c6 == GC_K8_BIG ? g.cand[v[k]] : (int)c6;
        ci[k] = x[k] >= 0 ? g.hcore[x[k]] : -1;
        const bool kill = x[k] >= 0 && g.hkill[x[k]] != 0u;
        if (x[k] < 0 || ci[k] < 0 || ci[k] >= cn || c6 == GC_K8_NONE || cand[k] < 0 || cand[k] > 0xFFFF) {
            bad = true;
            continue;
        }
        st[k] = kill ? GC_JP_OUT : GC_JP_UND;  // a light winner of its candidate that it lists: OUT
        if (!kill) {
            s_cc[ci[k]] = (unsigned short)cand[k];
            atomicOr(&s_und[ci[k] >> 5], 1u << (ci[k] & 31));
        }
    }
    if (bad) s_bad = 1;
    __syncthreads();
    if (s_bad) return;  // nothing written: k_sweep_async takes the round
#ifdef GC_A_PROF
    const ull tp1 = wall_clock64();
    const ull cp1 = clock64();
#endif
    const long long W = (cn + 31) / 32;
    int windows = 0;
    for (;;) {
        // 1. the window: the first CORE_WIN set bits of s_und (the lowest-rank undecided proposers),
        //    block-parallel: thread t < WMAX takes word t; a scan of the words' popcounts gives each
        //    word the rank of its first bit, and the words holding ranks < CORE_WIN list their bits
        int wcnt = 0, wexcl = 0;
        unsigned wdw = 0u;
        if (t < WMAX) {
            wdw = t < Wc ? s_und[t] : 0u;
            wcnt = __popc(wdw);
            const int incl = gc_wave_incl_scan(wcnt);
            if (lane == GC_WAVE - 1) s_wt[t / GC_WAVE] = incl;
            wexcl = incl - wcnt;
        }
        __syncthreads();
        int total = 0;
#pragma unroll
        for (int i = 0; i < WMAX / GC_WAVE; ++i) {
            if (i < t / GC_WAVE) wexcl += s_wt[i];
            total += s_wt[i];
        }
        if (t < WMAX && wcnt && wexcl < CORE_WIN) {
            int pos = wexcl;
            for (unsigned m = wdw; m && pos < CORE_WIN; m &= m - 1, ++pos) {
                const int cix = t * 32 + __builtin_ctz(m);
                s_win[pos] = cix;
                s_wpos[cix] = (unsigned char)pos;
            }
        }
        if (t < CORE_WIN) s_P[t] = 0ull;
        __syncthreads();
#ifdef GC_A_PROF
        if (t == 0 && windows == 0 && c->round < GC_C_PROF_ROUNDS) gc_tstep[c->round][1] = wall_clock64() - tp1;
#endif
        const int nw = total < CORE_WIN ? total : CORE_WIN;
        if (nw == 0) break;
        if (++windows > g.core_iters) {  // (tests: GC_HUB_CORE_ITERS forces the hand-over)
            s_bad = 2;
            break;
        }
        // 2. their bitsets into LDS (coalesced; wave w takes rows w, w + 16, w + 32, w + 48, its
        //    lanes 4 words of each: every load in flight before the first store)
        {
            constexpr int NWV = GC_CORE_BLOCK / GC_WAVE, RPW = CORE_WIN / NWV, KPR = WMAX / GC_WAVE;
            const int w = t / GC_WAVE;
            const unsigned* rowp[RPW];
#pragma unroll
            for (int rr = 0; rr < RPW; ++rr) {
                const int r = w + rr * NWV;
                rowp[rr] = r < nw ? g.core_bits + (long long)s_win[r] * W : nullptr;
            }
            unsigned val[RPW][KPR];
#pragma unroll
            for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
                for (int k = 0; k < KPR; ++k) {
                    const int wd = k * GC_WAVE + lane;
                    val[rr][k] = (rowp[rr] && wd < Wc) ? rowp[rr][wd] : 0u;
                }
#pragma unroll
            for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
                for (int k = 0; k < KPR; ++k) {
                    const int wd = k * GC_WAVE + lane;
                    if (rowp[rr] && wd < Wc) s_rows[w + rr * NWV][wd] = val[rr][k];
                }
        }
        __syncthreads();
#ifdef GC_A_PROF
        if (t == 0 && windows <= 1 && c->round < GC_C_PROF_ROUNDS) gc_tstep[c->round][2] = wall_clock64() - tp1;
#endif
        // 3. the window in rank order.  P_j = the earlier window members of j's class that j lists
        //    (bit cj in their bitsets): thread (j = t % 64, i-block t / 64) tests 4 of them.  Then
        //    wave 0 runs the JP on the window: a member whose predecessors are all decided is IN
        //    if none of them is IN, else OUT -- the greedy in rank order, its chain in ballots.
        {
            const int jj = t % CORE_WIN, ib = t / CORE_WIN;
            constexpr int IPB = CORE_WIN / (GC_CORE_BLOCK / CORE_WIN);
            if (jj < nw) {
                const int cj = s_win[jj];
                const unsigned ccj = s_cc[cj];
                ull part = 0;
#pragma unroll
                for (int q = 0; q < IPB; ++q) {
                    const int i = ib * IPB + q;
                    if (i < jj && s_cc[s_win[i]] == ccj && ((s_rows[i][cj >> 5] >> (cj & 31)) & 1u)) part |= 1ull << i;
                }
                if (part) atomicOr(&s_P[jj], part);
            }
        }
        __syncthreads();
        if (t < GC_WAVE) {
            const ull P = s_P[lane];
            ull und = nw == 64 ? ~0ull : ((1ull << nw) - 1ull), inm = 0;
            while (und) {
                const bool mine = (und >> lane) & 1ull;
                const bool ready = mine && !(P & und);
                const ull rdy = __ballot(ready), ins = __ballot(ready && !(P & inm));
                inm |= ins;
                und &= ~rdy;
            }
            if (lane == 0) s_inmask = inm;
        }
        __syncthreads();
#ifdef GC_A_PROF
        if (t == 0 && windows <= 1 && c->round < GC_C_PROF_ROUNDS) gc_tstep[c->round][3] = wall_clock64() - tp1;
#endif
        // 4. decisions: the window's members, and every proposer listing one of its class's winners
        const ull inm = s_inmask;
        const int last = s_win[nw - 1];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            if (st[k] != GC_JP_UND) continue;
            const int cix = ci[k];
            if (cix <= last) {  // in the window (every undecided index up to its last one is)
                st[k] = ((inm >> s_wpos[cix]) & 1ull) ? GC_JP_IN : GC_JP_OUT;
            } else {
                for (ull m = inm; m; m &= m - 1) {
                    const int r = __ffsll((long long)m) - 1;
                    if (s_cc[s_win[r]] == (unsigned)cand[k] && ((s_rows[r][cix >> 5] >> (cix & 31)) & 1u)) {
                        st[k] = GC_JP_OUT;
                        break;
                    }
                }
            }
            if (st[k] != GC_JP_UND) atomicAnd(&s_und[cix >> 5], ~(1u << (cix & 31)));
        }
        __syncthreads();
#ifdef GC_A_PROF
        if (t == 0 && windows <= 1 && c->round < GC_C_PROF_ROUNDS) gc_tstep[c->round][4] = wall_clock64() - tp1;
#endif
    }
    if (s_bad) return;  // GC_HUB_CORE_ITERS windows were not enough: nothing written, k_sweep_async decides
#ifdef GC_A_PROF
    if (c->round < GC_C_PROF_ROUNDS) {
        ull* prof = gc_cprof[c->round];
        ull win = 0, killed = 0;
        for (int k = 0; k < U; ++k) {
            win += (v[k] >= 0 && st[k] == GC_JP_IN) ? 1ull : 0ull;
        }
        (void)killed;
        if (win) atomicAdd(prof + 5, win);
        if (t == 0) {
            const ull tp2 = wall_clock64();
            prof[0] = (ull)n;
            prof[1] = tp1 - tp0;  // load + setup (10 ns ticks)
            prof[2] = tp2 - tp1;  // the windows
            prof[3] = (ull)(clock64() - cp1);  // shader clock cycles over the windows
            prof[4] = (ull)windows;
            prof[6] = 1ull;
        }
    }
#endif
    // the decisions, as k_sweep_async stores them (the commit reads k8, later rounds' scans hk)
#pragma unroll
    for (int k = 0; k < U; ++k) {
        if (v[k] < 0) continue;
        g.k8[v[k]] = gc_k8(gc_c6_of(cand[k]), st[k]);
        g.hk[x[k]] = gc_hk((unsigned)cand[k], st[k]);
    }
    if (t == 0) {  // k_sweep_async's bookkeeping for a launch that decided every hub
        c->und_cnt[z] = 0;
        c->undh_cnt[z] = 0;
        c->tail_last = j + 1;
        c->sweeps += 1;
        c->async_done[par ^ 1] = 0;
        c->async_abort[par ^ 1] = 0;
        c->hub_start = j + 1;
        c->core_round = c->round;
        c->core_handled += 1;
        c->core_iters_sum += windows;
        if (windows > c->core_iters_max) c->core_iters_max = windows;
    }
}

// ------------------------------------------------------------------------------------
// host
// ------------------------------------------------------------------------------------
void gcl_core_build(const GDev& g, hipStream_t s) {
    if (!g.core_cap || !g.hcore) return;
    hipMemsetAsync(&g.ctl->core_cnt, 0, sizeof(ull), s);
    const long long nhub = g.nhub_core;
    GC_LAUNCH(k_core_count, dim3(GC_CORE_BUILD_GRID), dim3(GC_BLOCK), 0, s, g, nhub);
    GC_LAUNCH(k_core_assign, dim3(GC_CORE_BUILD_GRID), dim3(GC_BLOCK), 0, s, g, nhub);
    GC_LAUNCH(k_core_zero, dim3(512), dim3(GC_BLOCK), 0, s, g);
    GC_LAUNCH(k_core_bits, dim3(1024), dim3(GC_BLOCK), 0, s, g);
}

void gcl_hub_core(const GDev& g, const GLists& L, int S, int par, hipStream_t s) {
    GC_LAUNCH(k_hub_core, dim3(1), dim3(GC_CORE_BLOCK), 0, s, g, L, S, par);
}

int gc_core_prepare(gc_graph* g, GDev& d) {
    d.core_cap = 0;
    // Opt-in (GC_HUB_CORE=1): bit-exact, but measured no faster than k_sweep_async alone --
    // R-MAT-24 154.58 vs 153.92 ms, R-MAT-26 426.7 vs 423.6 (interleaved, profiles/r06/b) -- see
    // DESIGN.md §13 for where its ~20 us per round go
    const char* e = getenv("GC_HUB_CORE");
    if (!e || atoi(e) == 0 || g->nhub <= 0) return GC_OK;
    int cap = GC_CORE_MAX;
    if (const char* ce = getenv("GC_HUB_CORE_CAP")) cap = std::max(1, std::min(cap, atoi(ce)));
    if (g->core_cap < GC_CORE_MAX) {  // buffers for the largest core, once per graph
        if (g->hcore) gc_dfree(g->hcore);
        if (g->core_hub) gc_dfree(g->core_hub);
        if (g->core_bits) gc_dfree(g->core_bits);
        if (g->core_wcnt) gc_dfree(g->core_wcnt);
        g->hcore = g->core_hub = nullptr;
        g->core_bits = nullptr;
        g->core_wcnt = nullptr;
        g->core_cap = 0;
        GC_HIP(gc_dmalloc((void**)&g->hcore, sizeof(int) * (size_t)g->nhub));
        GC_HIP(gc_dmalloc((void**)&g->core_hub, sizeof(int) * (size_t)GC_CORE_MAX));
        GC_HIP(gc_dmalloc((void**)&g->core_bits, sizeof(unsigned) * (size_t)GC_CORE_MAX * (GC_CORE_MAX / 32)));
        GC_HIP(gc_dmalloc((void**)&g->core_wcnt, sizeof(ull) * GC_CORE_BUILD_GRID));
        g->core_cap = GC_CORE_MAX;
    }
    d.hcore = g->hcore;
    d.core_hub = g->core_hub;
    d.core_bits = g->core_bits;
    d.core_wcnt = g->core_wcnt;
    d.nhub_core = g->nhub;
    d.core_cap = cap;
    d.core_iters = 1 << 20;  // windows a round may take (at most GC_CORE_MAX / 64 by construction)
    if (const char* ie = getenv("GC_HUB_CORE_ITERS")) d.core_iters = std::max(1, atoi(ie));
    return GC_OK;
}
