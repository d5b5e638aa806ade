// gc_kernels.hip -- gfx950 kernels of the colouring round (variant A, coloring.py:73-132).
//
// Per round r (host engine in gc_engine.hip drives the order):
//   propose  : k_propose_light (edge-balanced wave chunks) + k_propose_block (hubs / wide mex)
//              mex of coloured neighbours' colours, colours as at the round start
//              (coloring.py:44-54, 82-83, 98-102)
//   resolve  : k_resolve_light / k_resolve_block, then k_resolve_light over the undecided
//              list until empty -- Jones-Plassmann sweeps computing, per candidate colour,
//              the lexicographically-first maximal independent set under rank
//              (deg asc, pos asc) == coloring.py:56-70's stable-sorted greedy pass
//   commit   : k_commit_light / k_commit_block -- scatter accepted colours
//              (coloring.py:37-41, 114-127) and push the next frontier from the newly
//              coloured vertices through the in-neighbour lists (claim bitmap + LDS-staged
//              appends), so the next round touches only vertices that can propose.
// E1 re-seed (k_unc_compact, k_cc_hook, k_cc_best, k_cc_seeds) and the validator
// (k_validate, coloring.py:149-162) live here too.
//
// Edge-balanced wave chunks: a wave takes 64 list entries, prefix-sums their degrees and
// walks the concatenated edge range 64 slots at a time, so consecutive lanes read
// consecutive col[] entries and no lane idles on a short row (HBM-bound gather work; no
// MFMA involved).
#include "gc_internal.h"

struct GDev {
    int n;
    long long nnz;
    const long long* rp;
    const int* col;
    const int* deg;
    const long long* trp;  // in-neighbour CSR (== rp/col when symmetric)
    const int* tcol;
    int* color;
    int* cround;
    ull* key;
    unsigned char* jp;
    unsigned int* inF;
    DevCtl* ctl;
};

// ------------------------------------------------------------------------------------
// init: coloring.py:12-17 (+ argmax seed key for coloring.py:19-35)
// ------------------------------------------------------------------------------------
// Isolated vertices are coloured at init; when some OTHER vertex lists one of them
// (asymmetric input) it must push like a committed vertex, so it joins the seed list.
__global__ void __launch_bounds__(GC_BLOCK) k_init(GDev g, int* seed_light) {
    __shared__ ull scratch[GC_WAVES_PER_BLOCK];
    const int lane = gc_lane();
    ull best = 0, unc = 0;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v - lane < g.n; v += stride) {
        const bool valid = v < g.n;
        const int d = valid ? g.deg[v] : 0;
        const bool iso = valid && d == 0;
        if (valid) {
            g.color[v] = iso ? 0 : -1;
            g.cround[v] = iso ? 0 : -1;
            g.key[v] = GC_KEY_INVALID;
            g.jp[v] = GC_JP_UND;
            if (!iso) {
                unc++;
                const ull k = ((ull)d << 32) | (ull)v;
                best = k > best ? k : best;
            }
        }
        const bool push0 = iso && g.trp[v + 1] > g.trp[v];
        if (push0) {
            g.key[v] = gc_make_key(0, 0);
            g.jp[v] = GC_JP_IN;
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
    g.key[s] = gc_make_key(0, (unsigned)d);
    g.jp[s] = GC_JP_IN;
    atomicOr(&g.inF[s >> 5], 1u << (s & 31));
    if (d > GC_HEAVY_T) seed_heavy[atomicAdd(&g.ctl->seed_cnt[1], 1ull)] = s;
    else seed_light[atomicAdd(&g.ctl->seed_cnt[0], 1ull)] = s;
}

// ------------------------------------------------------------------------------------
// propose (assign_color, coloring.py:44-54)
// ------------------------------------------------------------------------------------
__global__ void __launch_bounds__(GC_BLOCK) k_propose_light(GDev g, const int* __restrict__ list,
                                                            const ull* list_cnt, int* heavy, int* wide,
                                                            long long kbound) {
    __shared__ ull s_mask[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ long long s_start[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ ull scratch[GC_WAVES_PER_BLOCK];
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    const long long cnt = (long long)*list_cnt;
    long long lmax = -1;
    ull lfail = 0, lsum = 0, lnv = 0;
    for (long long chunk = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w; chunk * GC_WAVE < cnt;
         chunk += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
        const long long idx = chunk * GC_WAVE + lane;
        const int v = idx < cnt ? list[idx] : -1;
        const int d = v >= 0 ? g.deg[v] : 0;
        const bool isheavy = d > GC_HEAVY_T;
        gc_wave_append(isheavy, v, heavy, &g.ctl->heavy_cnt);
        const int de = isheavy ? 0 : d;
        s_mask[w][lane] = 0;
        s_start[w][lane] = v >= 0 ? g.rp[v] : 0;
        const int incl = gc_wave_incl_scan(de);
        const int excl = incl - de;
        const int total = __shfl(incl, GC_WAVE - 1, GC_WAVE);
        gc_wave_sync();
        for (int base = 0; base < total; base += GC_WAVE) {
            const int e = base + lane;
            const int o = gc_owner(excl, e);
            const int eo = __shfl(excl, o, GC_WAVE);
            if (e < total) {
                const int u = g.col[s_start[w][o] + (e - eo)];
                const int c = g.color[u];
                if ((unsigned)c < 64u) atomicOr(&s_mask[w][o], 1ull << c);
            }
        }
        gc_wave_sync();
        bool iswide = false;
        if (v >= 0 && !isheavy) {
            const ull m = s_mask[w][lane];
            if (m == ~0ull) {
                iswide = true;
            } else {
                const int mex = __builtin_ctzll(~m);
                g.key[v] = gc_make_key((unsigned)mex, (unsigned)d);
                g.jp[v] = GC_JP_UND;
                lmax = mex > lmax ? mex : lmax;
                if (kbound >= 0 && mex >= kbound) lfail++;
                lsum += (ull)d;
                lnv++;
            }
        }
        gc_wave_append(iswide, v, wide, &g.ctl->wide_cnt);
    }
    __syncthreads();
    gc_block_max(&g.ctl->maxmex, lmax, (long long*)scratch);
    gc_block_add(&g.ctl->failcnt, lfail, scratch);
    gc_block_add(&g.ctl->sumdeg[1], lsum, scratch);
    gc_block_add(&g.ctl->nvert[1], lnv, scratch);
}

// One workgroup per vertex: hubs (deg > GC_HEAVY_T) and light vertices whose mex >= 64.
// Forbidden-colour bitmap in LDS covering [base, base + 32*words); mex <= maxcolor + 1,
// so one window suffices unless the colour count outgrows the LDS budget.
__global__ void __launch_bounds__(GC_BLOCK) k_propose_block(GDev g, const int* la, const ull* ca,
                                                            const int* lb, const ull* cb, long long kbound,
                                                            int words) {
    extern __shared__ __attribute__((aligned(16))) unsigned s_bits[];
    __shared__ int s_first;
    __shared__ ull scratch[GC_WAVES_PER_BLOCK];
    const long long na = (long long)*ca, nb = (long long)*cb;
    long long lmax = -1;
    ull lfail = 0, lsum = 0, lnv = 0;
    for (long long i = blockIdx.x; i < na + nb; i += gridDim.x) {
        const int v = i < na ? la[i] : lb[i - na];
        const int d = g.deg[v];
        const long long start = g.rp[v];
        long long mex = -1;
        for (long long base = 0; mex < 0; base += 32ll * words) {
            for (int t = threadIdx.x; t < words; t += blockDim.x) s_bits[t] = 0;
            if (threadIdx.x == 0) s_first = 0x7FFFFFFF;
            __syncthreads();
            for (long long e = threadIdx.x; e < d; e += blockDim.x) {
                const long long c = g.color[g.col[start + e]] - base;
                if (c >= 0 && c < 32ll * words) atomicOr(&s_bits[c >> 5], 1u << (c & 31));
            }
            __syncthreads();
            for (int t = threadIdx.x; t < words; t += blockDim.x)
                if (~s_bits[t]) atomicMin(&s_first, t);
            __syncthreads();
            if (s_first != 0x7FFFFFFF) mex = base + 32ll * s_first + __builtin_ctz(~s_bits[s_first]);
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            g.key[v] = gc_make_key((unsigned)mex, (unsigned)d);
            g.jp[v] = GC_JP_UND;
            lmax = mex > lmax ? mex : lmax;
            if (kbound >= 0 && mex >= kbound) lfail++;
            lsum += (ull)d;
            lnv++;
        }
    }
    __syncthreads();
    gc_block_max(&g.ctl->maxmex, lmax, (long long*)scratch);
    gc_block_add(&g.ctl->failcnt, lfail, scratch);
    gc_block_add(&g.ctl->sumdeg[1], lsum, scratch);
    gc_block_add(&g.ctl->nvert[1], lnv, scratch);
}

// ------------------------------------------------------------------------------------
// resolve (resolve_collisions, coloring.py:56-70) as Jones-Plassmann sweeps.
// v is IN iff every same-candidate listed neighbour u of lower rank is OUT, OUT as soon
// as one is IN.  States only move UND -> IN/OUT, so reading a newer state than the
// sweep started with is harmless (decisions are final).
// ------------------------------------------------------------------------------------
__global__ void __launch_bounds__(GC_BLOCK) k_resolve_light(GDev g, const int* __restrict__ list,
                                                            const ull* list_cnt, int skip_heavy,
                                                            int* und, ull* und_cnt, int kclass) {
    __shared__ unsigned s_flag[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ long long s_start[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_v[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ unsigned s_cand[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ unsigned s_deg[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ ull scratch[GC_WAVES_PER_BLOCK];
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    const long long cnt = (long long)*list_cnt;
    ull lsum = 0, lnv = 0;
    for (long long chunk = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w; chunk * GC_WAVE < cnt;
         chunk += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
        const long long idx = chunk * GC_WAVE + lane;
        const int v = idx < cnt ? list[idx] : -1;
        const int d = v >= 0 ? g.deg[v] : 0;
        const bool skip = v < 0 || (skip_heavy && d > GC_HEAVY_T);
        const int de = skip ? 0 : d;
        s_flag[w][lane] = 0;
        s_start[w][lane] = v >= 0 ? g.rp[v] : 0;
        s_v[w][lane] = v;
        s_cand[w][lane] = skip ? 0xFFFFFFFFu : gc_key_cand(g.key[v]);
        s_deg[w][lane] = (unsigned)d;
        const int incl = gc_wave_incl_scan(de);
        const int excl = incl - de;
        const int total = __shfl(incl, GC_WAVE - 1, GC_WAVE);
        gc_wave_sync();
        for (int base = 0; base < total; base += GC_WAVE) {
            const int e = base + lane;
            const int o = gc_owner(excl, e);
            const int eo = __shfl(excl, o, GC_WAVE);
            if (e < total) {
                const int u = g.col[s_start[w][o] + (e - eo)];
                const int vo = s_v[w][o];
                if (u != vo) {
                    const ull ku = g.key[u];
                    if (gc_key_cand(ku) == s_cand[w][o] && gc_rank_lt(gc_key_deg(ku), u, s_deg[w][o], vo)) {
                        const unsigned char st = g.jp[u];
                        if (st == GC_JP_IN) atomicOr(&s_flag[w][o], 1u);
                        else if (st == GC_JP_UND) atomicOr(&s_flag[w][o], 2u);
                    }
                }
            }
        }
        gc_wave_sync();
        bool pend = false;
        if (!skip) {
            const unsigned f = s_flag[w][lane];
            if (f & 1u) g.jp[v] = GC_JP_OUT;
            else if (f & 2u) pend = true;
            else g.jp[v] = GC_JP_IN;
            lsum += (ull)d;
            lnv++;
        }
        gc_wave_append(pend, v, und, und_cnt);
    }
    __syncthreads();
    gc_block_add(&g.ctl->sumdeg[kclass], lsum, scratch);
    gc_block_add(&g.ctl->nvert[kclass], lnv, scratch);
}

__global__ void __launch_bounds__(GC_BLOCK) k_resolve_block(GDev g, const int* list, const ull* list_cnt,
                                                            int* und, ull* und_cnt) {
    __shared__ unsigned s_f;
    __shared__ ull scratch[GC_WAVES_PER_BLOCK];
    const long long cnt = (long long)*list_cnt;
    ull lsum = 0, lnv = 0;
    for (long long i = blockIdx.x; i < cnt; i += gridDim.x) {
        const int v = list[i];
        const int d = g.deg[v];
        const long long start = g.rp[v];
        const unsigned cv = gc_key_cand(g.key[v]);
        if (threadIdx.x == 0) s_f = 0;
        __syncthreads();
        unsigned f = 0;
        for (long long e = threadIdx.x; e < d; e += blockDim.x) {
            const int u = g.col[start + e];
            if (u == v) continue;
            const ull ku = g.key[u];
            if (gc_key_cand(ku) == cv && gc_rank_lt(gc_key_deg(ku), u, (unsigned)d, v)) {
                const unsigned char st = g.jp[u];
                f |= st == GC_JP_IN ? 1u : (st == GC_JP_UND ? 2u : 0u);
            }
        }
        if (f) atomicOr(&s_f, f);
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned ff = s_f;
            if (ff & 1u) g.jp[v] = GC_JP_OUT;
            else if (ff & 2u) und[atomicAdd(und_cnt, 1ull)] = v;
            else g.jp[v] = GC_JP_IN;
            lsum += (ull)d;
            lnv++;
        }
        __syncthreads();
    }
    gc_block_add(&g.ctl->sumdeg[2], lsum, scratch);
    gc_block_add(&g.ctl->nvert[2], lnv, scratch);
}

// ------------------------------------------------------------------------------------
// commit (color_node + join, coloring.py:37-41, 114-127) fused with the frontier push.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ bool gc_claim(unsigned* inF, int w) {
    const unsigned bit = 1u << (w & 31);
    if (inF[w >> 5] & bit) return false;
    return !(atomicOr(&inF[w >> 5], bit) & bit);
}

__global__ void __launch_bounds__(GC_BLOCK) k_commit_light(GDev g, const int* __restrict__ list,
                                                           const ull* list_cnt, int skip_heavy, int* next,
                                                           ull* next_cnt, int round) {
    __shared__ int s_stage[GC_WAVES_PER_BLOCK][GC_STAGE_CAP];
    __shared__ long long s_start[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ ull scratch[GC_WAVES_PER_BLOCK];
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    const long long cnt = (long long)*list_cnt;
    GcStage st{s_stage[w], 0};
    long long lmaxc = -1;
    ull lacc = 0, lsum = 0;
    for (long long chunk = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w; chunk * GC_WAVE < cnt;
         chunk += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
        const long long idx = chunk * GC_WAVE + lane;
        const int v = idx < cnt ? list[idx] : -1;
        const int d = v >= 0 ? g.deg[v] : 0;
        const bool skip = v < 0 || (skip_heavy && d > GC_HEAVY_T);
        const unsigned char js = skip ? GC_JP_UND : g.jp[v];
        const bool acc = js == GC_JP_IN;
        int din = 0;
        long long tstart = 0;
        if (acc) {
            const int c = (int)gc_key_cand(g.key[v]);
            g.color[v] = c;
            g.cround[v] = round;
            g.key[v] = GC_KEY_INVALID;
            lmaxc = c > lmaxc ? c : lmaxc;
            lacc++;
            tstart = g.trp[v];
            din = (int)(g.trp[v + 1] - tstart);
            lsum += (ull)din;
        }
        // losers stay in the frontier (they still have a coloured neighbour)
        gc_stage_push(st, js == GC_JP_OUT, v, next, next_cnt);
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
    }
    gc_stage_flush(st, next, next_cnt);
    __syncthreads();
    gc_block_max(&g.ctl->maxcolor, lmaxc, (long long*)scratch);
    gc_block_add(&g.ctl->accepted, lacc, scratch);
    gc_block_add(&g.ctl->sumdeg[4], lsum, scratch);
    gc_block_add(&g.ctl->nvert[4], lacc, scratch);
}

__global__ void __launch_bounds__(GC_BLOCK) k_commit_block(GDev g, const int* list, const ull* list_cnt,
                                                           int* next, ull* next_cnt, int round) {
    __shared__ int s_stage[GC_WAVES_PER_BLOCK][GC_STAGE_CAP];
    __shared__ int s_acc;
    __shared__ ull scratch[GC_WAVES_PER_BLOCK];
    const int w = threadIdx.x / GC_WAVE;
    const long long cnt = (long long)*list_cnt;
    GcStage st{s_stage[w], 0};
    long long lmaxc = -1;
    ull lacc = 0, lsum = 0;
    for (long long i = blockIdx.x; i < cnt; i += gridDim.x) {
        const int v = list[i];
        if (threadIdx.x == 0) {
            const unsigned char js = g.jp[v];
            s_acc = js == GC_JP_IN;
            if (js == GC_JP_IN) {
                const int c = (int)gc_key_cand(g.key[v]);
                g.color[v] = c;
                g.cround[v] = round;
                g.key[v] = GC_KEY_INVALID;
                lmaxc = c > lmaxc ? c : lmaxc;
                lacc++;
                lsum += (ull)(g.trp[v + 1] - g.trp[v]);
            } else if (js == GC_JP_OUT) {
                next[atomicAdd(next_cnt, 1ull)] = v;
            }
        }
        __syncthreads();
        if (s_acc) {
            const long long ts = g.trp[v], te = g.trp[v + 1];
            for (long long e0 = ts; e0 < te; e0 += blockDim.x) {
                const long long e = e0 + threadIdx.x;
                bool claim = false;
                int x = 0;
                if (e < te) {
                    x = g.tcol[e];
                    claim = gc_claim(g.inF, x);
                }
                gc_stage_push(st, claim, x, next, next_cnt);
            }
        }
        __syncthreads();
    }
    gc_stage_flush(st, next, next_cnt);
    __syncthreads();
    gc_block_max(&g.ctl->maxcolor, lmaxc, (long long*)scratch);
    gc_block_add(&g.ctl->accepted, lacc, scratch);
    gc_block_add(&g.ctl->sumdeg[4], lsum, scratch);
    gc_block_add(&g.ctl->nvert[4], lacc, scratch);
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
    GcStage st{s_stage[w], 0};
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v - lane < g.n; v += stride) {
        const bool u = v < g.n && g.color[v] == -1;
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
                if (u != a && g.color[u] == -1) {
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
            g.key[s] = gc_make_key(0, (unsigned)d);
            g.jp[s] = GC_JP_IN;
            atomicOr(&g.inF[s >> 5], 1u << (s & 31));
        }
        gc_wave_append(root && d > GC_HEAVY_T, s, seed_heavy, &g.ctl->seed_cnt[1]);
        gc_wave_append(root && d <= GC_HEAVY_T, s, seed_light, &g.ctl->seed_cnt[0]);
    }
}

// ------------------------------------------------------------------------------------
// validate_graph_coloring counts (coloring.py:149-162)
// ------------------------------------------------------------------------------------
__global__ void __launch_bounds__(GC_BLOCK) k_validate(GDev g, const int* __restrict__ colors) {
    __shared__ long long s_start[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ int s_c[GC_WAVES_PER_BLOCK][GC_WAVE];
    __shared__ ull scratch[GC_WAVES_PER_BLOCK];
    const int lane = gc_lane();
    const int w = threadIdx.x / GC_WAVE;
    ull unc = 0, conf = 0;
    const long long nchunks = ((long long)g.n + GC_WAVE - 1) / GC_WAVE;
    for (long long chunk = (long long)blockIdx.x * GC_WAVES_PER_BLOCK + w; chunk < nchunks;
         chunk += (long long)gridDim.x * GC_WAVES_PER_BLOCK) {
        const long long v = chunk * GC_WAVE + lane;
        const bool valid = v < g.n;
        const int d = valid ? g.deg[v] : 0;
        const int c = valid ? colors[v] : 0;
        if (valid && c == -1) unc++;
        s_start[w][lane] = valid ? g.rp[v] : 0;
        s_c[w][lane] = c;
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
                if (colors[u] == s_c[w][o]) conf++;
            }
        }
        gc_wave_sync();
    }
    __syncthreads();
    gc_block_add(&g.ctl->uncolored, unc, scratch);
    gc_block_add(&g.ctl->conflicts, conf, scratch);
}

// ------------------------------------------------------------------------------------
// graph helpers
// ------------------------------------------------------------------------------------
__global__ void k_degrees(const long long* rp, int n, int* deg, ull* maxdeg) {
    ull m = 0;
    for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (long long)gridDim.x * blockDim.x) {
        const long long d = rp[v + 1] - rp[v];
        deg[v] = (int)d;
        m = (ull)d > m ? (ull)d : m;
    }
    m = gc_wave_max(m);
    if (gc_lane() == 0 && m) atomicMax(maxdeg, m);
}

// ------------------------------------------------------------------------------------
// host-callable launch wrappers (extern "C++" linkage within the library)
// ------------------------------------------------------------------------------------
#include "gc_launch.h"

static inline GDev to_dev(const GcDevView& d) {
    GDev g;
    g.n = d.n; g.nnz = d.nnz; g.rp = d.rp; g.col = d.col; g.deg = d.deg; g.trp = d.trp; g.tcol = d.tcol;
    g.color = d.color; g.cround = d.cround; g.key = d.key; g.jp = d.jp; g.inF = d.inF; g.ctl = d.ctl;
    return g;
}

void gcl_init(const GcDevView& d, int* seed_light, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_init, dim3(grid), dim3(GC_BLOCK), 0, s, to_dev(d), seed_light);
}
void gcl_seed_prep(const GcDevView& d, int* sl, int* sh, hipStream_t s) {
    hipLaunchKernelGGL(k_seed_prep, dim3(1), dim3(64), 0, s, to_dev(d), sl, sh);
}
void gcl_propose_light(const GcDevView& d, const int* list, const ull* cnt, int* heavy, int* wide, long long k,
                       int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_propose_light, dim3(grid), dim3(GC_BLOCK), 0, s, to_dev(d), list, cnt, heavy, wide, k);
}
void gcl_propose_block(const GcDevView& d, const int* la, const ull* ca, const int* lb, const ull* cb, long long k,
                       int words, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_propose_block, dim3(grid), dim3(GC_BLOCK), (size_t)words * 4, s, to_dev(d), la, ca, lb, cb,
                       k, words);
}
void gcl_resolve_light(const GcDevView& d, const int* list, const ull* cnt, int skip_heavy, int* und, ull* und_cnt,
                       int kclass, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_resolve_light, dim3(grid), dim3(GC_BLOCK), 0, s, to_dev(d), list, cnt, skip_heavy, und,
                       und_cnt, kclass);
}
void gcl_resolve_block(const GcDevView& d, const int* list, const ull* cnt, int* und, ull* und_cnt, int grid,
                       hipStream_t s) {
    hipLaunchKernelGGL(k_resolve_block, dim3(grid), dim3(GC_BLOCK), 0, s, to_dev(d), list, cnt, und, und_cnt);
}
void gcl_commit_light(const GcDevView& d, const int* list, const ull* cnt, int skip_heavy, int* next, ull* next_cnt,
                      int round, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_commit_light, dim3(grid), dim3(GC_BLOCK), 0, s, to_dev(d), list, cnt, skip_heavy, next,
                       next_cnt, round);
}
void gcl_commit_block(const GcDevView& d, const int* list, const ull* cnt, int* next, ull* next_cnt, int round,
                      int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_commit_block, dim3(grid), dim3(GC_BLOCK), 0, s, to_dev(d), list, cnt, next, next_cnt, round);
}
void gcl_unc_compact(const GcDevView& d, int* list, ull* cnt, int* parent, ull* best, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_unc_compact, dim3(grid), dim3(GC_BLOCK), 0, s, to_dev(d), list, cnt, parent, best);
}
void gcl_cc_hook(const GcDevView& d, const int* list, const ull* cnt, int* parent, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_cc_hook, dim3(grid), dim3(GC_BLOCK), 0, s, to_dev(d), list, cnt, parent);
}
void gcl_cc_best(const GcDevView& d, const int* list, const ull* cnt, int* parent, ull* best, int grid,
                 hipStream_t s) {
    hipLaunchKernelGGL(k_cc_best, dim3(grid), dim3(GC_BLOCK), 0, s, to_dev(d), list, cnt, parent, best);
}
void gcl_cc_seeds(const GcDevView& d, const int* list, const ull* cnt, int* parent, const ull* best, int* sl,
                  int* sh, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_cc_seeds, dim3(grid), dim3(GC_BLOCK), 0, s, to_dev(d), list, cnt, parent, best, sl, sh);
}
void gcl_validate(const GcDevView& d, const int* colors, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_validate, dim3(grid), dim3(GC_BLOCK), 0, s, to_dev(d), colors);
}
void gcl_degrees(const long long* rp, int n, int* deg, ull* maxdeg, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_degrees, dim3(grid), dim3(GC_BLOCK), 0, s, rp, n, deg, maxdeg);
}
