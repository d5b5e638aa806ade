// gc_hubs.hip -- push-maintained state of the high-degree vertices (variant A, one GPU).
//
// On power-law graphs (R-MAT) the rank (deg, pos) of coloring.py:64 puts hubs last: a hub
// loses round after round and stays in the frontier for hundreds of rounds.  Done as the
// reference states it, every one of those rounds re-reads the hub's whole row twice --
// assign_color's set of neighbour colours (coloring.py:44-54) and resolve_collisions'
// same-colour check (coloring.py:56-70) -- and the JP sweeps re-read the low part again
// per sweep: on R-MAT-24 that is ~40x nnz of gathers.  Hubs (deg > heavy_t) instead keep
// the two facts those reads establish, and the low-degree side pushes them:
//   hbits  forbidden-colour bitmap: when u is coloured c (any commit: seed, round, E1),
//          u sets bit c in every hub that lists u (hin = the hub-restricted transpose).
//          The hub's mex is the first zero bit -- the same value as the mex of its coloured
//          neighbours' colours, because the bitmap holds exactly those colours (< 4096;
//          beyond that the hub falls back to the row scan).
//   hkill  conflict resolution: a light vertex's low row holds only light vertices (every
//          hub ranks above it), so the lights' Jones-Plassmann sweeps never wait on a hub.
//          Hubs therefore sit out the sweeps until the lights have converged; a light that
//          decides IN flags every hub that lists it and proposes its candidate (hkill, via
//          its hin row).  Then a hub is OUT if flagged, and otherwise runs JP against the
//          lower-rank HUBS of its row only (hlow, built once): exactly the LFMIS rule of
//          coloring.py:56-70 over its whole low row, because every light entry is decided
//          by then and the flag says whether one of them won the same colour.
// Both are sets and flags: the order of pushes cannot change a mex or a JP decision, so
// results stay bit-identical to the row-scan engine (and to the oracle).  The cost moves
// to the low-degree side -- one walk of a vertex's hin row when it is coloured (bitmaps)
// and one when it wins (flags) -- instead of every hub re-reading its row every round.
#include <chrono>
#include <numeric>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <rocprim/rocprim.hpp>

#include "gc_device.h"
#include "gc_engine.h"

namespace {

// hub bitmap (bit per vertex: deg > T) by ballot, and its per-word counts
__global__ void k_hub_bits(const int* deg, long long n, int T, unsigned* map, unsigned* wcnt) {
    const long long words = (n + 31) / 32;
    for (long long v0 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) & ~63ll; v0 < n;
         v0 += (long long)gridDim.x * blockDim.x) {
        const long long v = v0 + gc_lane();
        const ull m = __ballot(v < n && deg[v] > T);
        const long long w = v0 >> 5;
        if (gc_lane() == 0) {
            map[w] = (unsigned)m;
            wcnt[w] = __popc((unsigned)m);
        } else if (gc_lane() == 32 && w + 1 < words) {
            map[w + 1] = (unsigned)(m >> 32);
            wcnt[w + 1] = __popc((unsigned)(m >> 32));
        }
    }
}

// the hubs in vertex order (id-order index = hubpre[w] + rank within the word); hid = -1 elsewhere
__global__ void k_hub_ids(long long n, const unsigned* map, const unsigned* pre, int* hid, int* hub_v) {
    for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (long long)gridDim.x * blockDim.x) {
        const unsigned m = map[v >> 5];
        const unsigned bit = 1u << (v & 31);
        hid[v] = -1;
        if (m & bit) hub_v[pre[v >> 5] + __popc(m & (bit - 1u))] = (int)v;
    }
}

// hub indices in rank order (deg, pos) -- the rank of coloring.py:64 -- so that an hlow
// row sorted by hub index lists its lower-rank hubs lowest rank first (gc_hub_scan_wave)
__global__ void k_hub_keys(const int* deg, const int* hub_v, long long H, ull* keys) {
    for (long long x = (long long)blockIdx.x * blockDim.x + threadIdx.x; x < H; x += (long long)gridDim.x * blockDim.x) {
        const int v = hub_v[x];
        keys[x] = ((ull)(unsigned)deg[v] << 32) | (ull)(unsigned)v;
    }
}
__global__ void k_hub_reindex(const ull* keys, long long H, int* hid, int* hub_v, const unsigned* map,
                              const unsigned* pre, int* hperm) {
    for (long long x = (long long)blockIdx.x * blockDim.x + threadIdx.x; x < H; x += (long long)gridDim.x * blockDim.x) {
        const int v = (int)(keys[x] & 0xFFFFFFFFull);
        hub_v[x] = v;
        hid[v] = (int)x;
        const unsigned bit = 1u << (v & 31);
        hperm[pre[v >> 5] + __popc(map[v >> 5] & (bit - 1u))] = (int)x;  // id-order index -> hub index
    }
}

// one wave per hub row
__global__ void k_hub_count(const long long* rp, const int* col, const int* hub_v, long long H, ull* cnt) {
    const long long waves = (long long)gridDim.x * (blockDim.x / GC_WAVE);
    for (long long x = (long long)blockIdx.x * (blockDim.x / GC_WAVE) + threadIdx.x / GC_WAVE; x < H; x += waves) {
        const int h = hub_v[x];
        for (long long e = rp[h] + gc_lane(); e < rp[h + 1]; e += GC_WAVE) atomicAdd(&cnt[col[e]], 1ull);
    }
}

__global__ void k_hub_fill(const long long* rp, const int* col, const int* hub_v, long long H, const long long* hin_rp,
                           ull* cursor, int* hin_col) {
    const long long waves = (long long)gridDim.x * (blockDim.x / GC_WAVE);
    for (long long x = (long long)blockIdx.x * (blockDim.x / GC_WAVE) + threadIdx.x / GC_WAVE; x < H; x += waves) {
        const int h = hub_v[x];
        for (long long e = rp[h] + gc_lane(); e < rp[h + 1]; e += GC_WAVE) {
            const int u = col[e];
            hin_col[hin_rp[u] + (long long)atomicAdd(&cursor[u], 1ull)] = (int)x;
        }
    }
}

// hub x's low row restricted to hubs: count, then fill (wave per hub, ballot compaction)
__global__ void k_hlow_count(const long long* rp, const int* col, const int* nlow, const int* hid, const int* hub_v,
                             long long H, long long* cnt) {
    const long long waves = (long long)gridDim.x * (blockDim.x / GC_WAVE);
    for (long long x = (long long)blockIdx.x * (blockDim.x / GC_WAVE) + threadIdx.x / GC_WAVE; x < H; x += waves) {
        const int h = hub_v[x];
        long long k = 0;
        for (long long e = rp[h] + gc_lane(); e < rp[h] + nlow[h]; e += GC_WAVE) k += hid[col[e]] >= 0;
        k = gc_wave_sum(k);
        if (gc_lane() == 0) cnt[x] = k;
    }
}

__global__ void k_hlow_fill(const long long* rp, const int* col, const int* nlow, const int* hid, const int* hub_v,
                            long long H, const long long* hlow_rp, int* hlow_col) {
    const long long waves = (long long)gridDim.x * (blockDim.x / GC_WAVE);
    for (long long x = (long long)blockIdx.x * (blockDim.x / GC_WAVE) + threadIdx.x / GC_WAVE; x < H; x += waves) {
        const int h = hub_v[x];
        long long o = hlow_rp[x];
        const long long e1 = rp[h] + nlow[h];
        for (long long e0 = rp[h]; e0 < e1; e0 += GC_WAVE) {
            const long long e = e0 + gc_lane();
            const int u = e < e1 ? col[e] : 0;
            const int hu = e < e1 ? hid[u] : -1;
            const bool p = hu >= 0;
            const ull m = __ballot(p);
            if (p) hlow_col[o + __popcll(m & gc_lanemask_lt())] = hu;  // hub index (mirror hk)
            o += __popcll(m);
        }
    }
}

// static chunks of the hlow rows: ceil(len / GC_HCH) per hub, then chunk -> hub
__global__ void k_hch_count(const long long* hlow_rp, long long H, long long* cnt) {
    const long long x = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (x < H) cnt[x] = (hlow_rp[x + 1] - hlow_rp[x] + GC_HCH - 1) / GC_HCH;
    else if (x == H) cnt[x] = 0;
}
__global__ void k_hch_fill(const long long* hch_rp, long long H, int* own) {
    const long long x = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (x < H)
        for (long long j = hch_rp[x]; j < hch_rp[x + 1]; ++j) own[j] = (int)x;
}

int scan_ll(const long long* in, long long* out, long long count, hipStream_t s) {
    size_t bytes = 0;
    GC_HIP(rocprim::exclusive_scan(nullptr, bytes, in, out, 0ll, (size_t)count, rocprim::plus<long long>(), s));
    void* tmp = nullptr;
    GC_HIP(gc_dmalloc(&tmp, bytes ? bytes : 1));
    hipError_t e = rocprim::exclusive_scan(tmp, bytes, in, out, 0ll, (size_t)count, rocprim::plus<long long>(), s);
    const hipError_t se = hipStreamSynchronize(s);  // (a fault of an earlier kernel on s shows here)
    gc_dfree(tmp);
    GC_HIP(e);
    GC_HIP(se);
    return GC_OK;
}

int scan_u32(const unsigned* in, unsigned* out, long long count, hipStream_t s) {
    size_t bytes = 0;
    GC_HIP(rocprim::exclusive_scan(nullptr, bytes, in, out, 0u, (size_t)count, rocprim::plus<unsigned>(), s));
    void* tmp = nullptr;
    GC_HIP(gc_dmalloc(&tmp, bytes ? bytes : 1));
    hipError_t e = rocprim::exclusive_scan(tmp, bytes, in, out, 0u, (size_t)count, rocprim::plus<unsigned>(), s);
    const hipError_t se = hipStreamSynchronize(s);
    gc_dfree(tmp);
    GC_HIP(e);
    GC_HIP(se);
    return GC_OK;
}

int grid_of(long long items) {
    return (int)std::max<long long>(1, std::min<long long>((items + GC_BLOCK - 1) / GC_BLOCK, 8192));
}

// threshold from GC_HUB_T ("off" or < 0 disables), default GC_HUB_T; GC_HUB_W sizes the
// bitmaps (tests shrink it to reach the row-scan fallback)
int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    if (!e || !*e) return dflt;
    if (strcmp(e, "off") == 0) return -1;
    return atoi(e);
}

// GC_PREP_TIMING=1: host-side phase times of the hub build on stderr (each phase ends in a
// stream synchronisation)
struct PhaseClock {
    bool on = getenv("GC_PREP_TIMING") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(const char* what, hipStream_t s) {
        if (!on) return;
        hipStreamSynchronize(s);
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[gc hubs] %-14s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
};

int build(gc_graph* g, int T, int W) {
    PhaseClock pc;
    hipStream_t s = g->stream;
    const long long n = g->n;
    // hub bitmap + per-word prefix counts (the hub transpose resolves an entry's hub index
    // from them: 2 + 2 MB on R-MAT-24 against the 67 MB hid array)
    const long long words = (n + 31) / 32;
    if (!g->hubmap) GC_HIP(gc_dmalloc((void**)&g->hubmap, sizeof(unsigned) * (size_t)std::max<long long>(words, 1)));
    GC_HIP(gc_dmalloc((void**)&g->hubpre, sizeof(unsigned) * (size_t)(words + 1)));
    unsigned* wcnt = nullptr;
    GC_HIP(gc_dmalloc((void**)&wcnt, sizeof(unsigned) * (size_t)(words + 1)));
    GC_HIP(hipMemsetAsync(wcnt + words, 0, sizeof(unsigned), s));
    hipLaunchKernelGGL(k_hub_bits, dim3(grid_of(n)), dim3(GC_BLOCK), 0, s, g->deg, n, T, g->hubmap, wcnt);
    int rc = scan_u32(wcnt, g->hubpre, words + 1, s);
    gc_dfree(wcnt);
    unsigned Hu = 0;
    if (!rc) rc = gc_read_dev(s, &Hu, (const unsigned*)g->hubpre + words);
    const long long H = Hu;
    long long* pos = nullptr;
    if (rc || H == 0) {
        g->hub_t = T;
        g->nhub = 0;
        return rc;
    }
    // memory: hid/hub_v, the hub transpose (one entry per hub-row entry), bitmaps, blockers
    size_t freeb = 0, totalb = 0;
    hipMemGetInfo(&freeb, &totalb);
    freeb += gc_cache_idle_bytes();
    const double need = 4.0 * (double)n + 8.0 * (double)(n + 1) + (28.0 + 4.0 * W) * (double)H;
    if (need > 0.5 * (double)freeb) {  // no room: row scans as before
        fprintf(stderr, "[gcolor] warning: hub index skipped (%lld hubs): its ids and bitmaps need %.1f GB, %.1f GB "
                        "free; hubs are resolved by row scans (slower)\n", H, need / 1e9, (double)freeb / 1e9);
        g->hub_t = T;
        g->nhub = 0;
        return GC_OK;
    }
    g->nhub = H;
    GC_HIP(gc_dmalloc((void**)&pos, sizeof(long long) * (size_t)(n + 1)));
    GC_HIP(gc_dmalloc((void**)&g->hid, sizeof(int) * (size_t)std::max<long long>(n, 1)));
    GC_HIP(gc_dmalloc((void**)&g->hub_v, sizeof(int) * (size_t)H));
    GC_HIP(gc_dmalloc((void**)&g->hperm, sizeof(int) * (size_t)H));
    hipLaunchKernelGGL(k_hub_ids, dim3(grid_of(n)), dim3(GC_BLOCK), 0, s, n, (const unsigned*)g->hubmap,
                       (const unsigned*)g->hubpre, g->hid, g->hub_v);
    pc.mark("bitmap+ids", s);
    {  // re-index the hubs in rank order
        ull *k0 = nullptr, *k1 = nullptr;
        GC_HIP(gc_dmalloc((void**)&k0, sizeof(ull) * (size_t)H));
        GC_HIP(gc_dmalloc((void**)&k1, sizeof(ull) * (size_t)H));
        hipLaunchKernelGGL(k_hub_keys, dim3(grid_of(H)), dim3(GC_BLOCK), 0, s, g->deg, g->hub_v, H, k0);
        size_t bytes = 0;
        GC_HIP(rocprim::radix_sort_keys(nullptr, bytes, k0, k1, (size_t)H, 0, 64, s));
        void* tmp = nullptr;
        GC_HIP(gc_dmalloc(&tmp, bytes ? bytes : 1));
        const hipError_t e = rocprim::radix_sort_keys(tmp, bytes, k0, k1, (size_t)H, 0, 64, s);
        if (e == hipSuccess)
            hipLaunchKernelGGL(k_hub_reindex, dim3(grid_of(H)), dim3(GC_BLOCK), 0, s, (const ull*)k1, H, g->hid, g->hub_v,
                               (const unsigned*)g->hubmap, (const unsigned*)g->hubpre, g->hperm);
        const hipError_t se = hipStreamSynchronize(s);
        gc_dfree(tmp);
        gc_dfree(k0);
        gc_dfree(k1);
        GC_HIP(e);
        GC_HIP(se);
    }
    pc.mark("rank sort", s);
    const int hgrid = (int)std::max<long long>(1, std::min<long long>((H + 3) / 4, 8192));
    long long E = 0, EL = 0;
    const bool sym = (g->flags & GC_GRAPH_SYMMETRIC) != 0;
    long long* klow = nullptr;
    GC_HIP(gc_dmalloc((void**)&g->hin_rp, sizeof(long long) * (size_t)(n + 1)));
    if (sym) {
        // symmetric: every row filtered for its hub entries (gc_prep.hip, a rank structure over
        // the entries): hin_rp directly, each hub row's lower-rank hubs (a prefix of its hin
        // row) into klow
        GC_HIP(gc_dmalloc((void**)&klow, sizeof(long long) * (size_t)(H + 1)));
        if ((rc = gc_hub_transpose_sym(g, H, g->hin_rp, klow, T))) { gc_dfree(pos); gc_dfree(klow); return rc; }
    } else {
        // hub transpose: reuse pos as the per-target counter
        GC_HIP(hipMemsetAsync(pos, 0, sizeof(long long) * (size_t)(n + 1), s));
        hipLaunchKernelGGL(k_hub_count, dim3(hgrid), dim3(GC_BLOCK), 0, s, g->rp, g->col, g->hub_v, H, (ull*)pos);
        if ((rc = scan_ll(pos, g->hin_rp, n + 1, s))) { gc_dfree(pos); return rc; }
    }
    GC_READ(s, &E, (const long long*)g->hin_rp + n, 1);
    GC_HIP(gc_dmalloc((void**)&g->hlow_rp, sizeof(long long) * (size_t)(H + 1)));
    if (sym) {  // the hlow rows' offsets now: their total sizes the memory check below
        rc = scan_ll(klow, g->hlow_rp, H + 1, s);
        gc_dfree(klow);
        klow = nullptr;
        if (rc) { gc_dfree(pos); return rc; }
        GC_READ(s, &EL, (const long long*)g->hlow_rp + H, 1);
    }
    pc.mark("hin count", s);
    hipMemGetInfo(&freeb, &totalb);
    freeb += gc_cache_idle_bytes();
    // hin (4 B per hub entry) + the hlow row and its four working copies (20 B per hlow entry;
    // symmetric graphs know EL here, others bound it by E).  Round 3's bound, 24 B per hub
    // entry, turned the hubs off for R-MAT-28 next to a resident CSR copy (the bench's step):
    // 49 s a step with row scans (profiles/r04/u).
    const double need2 = 4.0 * (double)E + 20.0 * (double)(sym ? EL : E) + (28.0 + 4.0 * W) * (double)H;
    if (need2 > 0.6 * (double)freeb) {
        fprintf(stderr, "[gcolor] warning: hub index skipped (%lld hubs, %lld hub entries): its transpose needs "
                        "%.1f GB, %.1f GB free; hubs are resolved by row scans (slower)\n", H, E, need2 / 1e9,
                (double)freeb / 1e9);
        gc_dfree(pos);
        gc_dfree(klow);
        gc_hub_bits_free(g);
        gc_hubs_free(g);
        g->hub_t = T;
        g->nhub = 0;
        return GC_OK;
    }
    GC_HIP(gc_dmalloc((void**)&g->hin_col, sizeof(int) * (size_t)std::max<long long>(E, 1)));
    GC_HIP(gc_dmalloc((void**)&g->hbits, sizeof(unsigned) * (size_t)H * W));
    GC_HIP(gc_dmalloc((void**)&g->hkill, sizeof(unsigned) * (size_t)H));
    GC_HIP(gc_dmalloc((void**)&g->hcur, sizeof(int) * (size_t)H));
    GC_HIP(gc_dmalloc((void**)&g->hpc, sizeof(int) * (size_t)H));
    if (!sym) {
        GC_HIP(hipMemsetAsync(pos, 0, sizeof(long long) * (size_t)(n + 1), s));
        hipLaunchKernelGGL(k_hub_fill, dim3(hgrid), dim3(GC_BLOCK), 0, s, g->rp, g->col, g->hub_v, H, g->hin_rp,
                           (ull*)pos, g->hin_col);
        // lower-rank hubs of each hub row (pos reused: H + 1 counts)
        GC_HIP(hipMemsetAsync(pos, 0, sizeof(long long) * (size_t)(H + 1), s));
        hipLaunchKernelGGL(k_hlow_count, dim3(hgrid), dim3(GC_BLOCK), 0, s, g->rp, g->col, g->nlow, g->hid, g->hub_v,
                           H, pos);
        if ((rc = scan_ll(pos, g->hlow_rp, H + 1, s))) { gc_dfree(pos); return rc; }
    }
    GC_READ(s, &EL, (const long long*)g->hlow_rp + H, 1);
    GC_HIP(gc_dmalloc((void**)&g->hlow_col, sizeof(int) * (size_t)std::max<long long>(EL, 1)));
    GC_HIP(gc_dmalloc((void**)&g->hpend[0], sizeof(int) * (size_t)std::max<long long>(EL, 1)));
    GC_HIP(gc_dmalloc((void**)&g->hpend[1], sizeof(int) * (size_t)std::max<long long>(EL, 1)));
    GC_HIP(gc_dmalloc((void**)&g->hlow2[0], sizeof(int) * (size_t)std::max<long long>(EL, 1)));
    GC_HIP(gc_dmalloc((void**)&g->hlow2[1], sizeof(int) * (size_t)std::max<long long>(EL, 1)));
    GC_HIP(gc_dmalloc((void**)&g->hrow, sizeof(int) * (size_t)H));
    GC_HIP(gc_dmalloc((void**)&g->hlen, sizeof(int) * (size_t)H));
    if (sym) {
        if ((rc = gc_hub_transpose_fill(g, H))) { gc_dfree(pos); return rc; }
    } else {
        hipLaunchKernelGGL(k_hlow_fill, dim3(hgrid), dim3(GC_BLOCK), 0, s, g->rp, g->col, g->nlow, g->hid, g->hub_v,
                           H, g->hlow_rp, g->hlow_col);
    }
    pc.mark("hin fill", s);
    // (Round 4 measured the rows left in row order: the scan's result does not depend on the
    // order, but rank order is what makes its coloured prefix (hlen) grow -- lower-rank hubs
    // colour first -- and the resumable scans skip it: unsorted, R-MAT-24 153.9 ms -> 6.0 s,
    // R-MAT-26 0.43 -> 25.9 s, profiles/r04/l.  The sort stays.)
    if (EL > 0) {  // every hlow row sorted by hub index == rank (gc_hub_scan_wave walks it in rank order)
        // the keys are hub indices < H: only their low bit_width(H - 1) bits are sorted
        // (R-MAT-26: 20 of 32 bits, three 8-bit digit passes instead of four)
        const unsigned kbits = (unsigned)std::max(1, 64 - __builtin_clzll((unsigned long long)std::max(H - 1, 1ll)));
        size_t bytes = 0;
        GC_HIP(rocprim::segmented_radix_sort_keys(nullptr, bytes, g->hlow_col, g->hpend[0], (unsigned)EL, (unsigned)H,
                                                  g->hlow_rp, g->hlow_rp + 1, 0, kbits, s));
        void* tmp = nullptr;
        GC_HIP(gc_dmalloc(&tmp, bytes ? bytes : 1));
        const hipError_t e = rocprim::segmented_radix_sort_keys(tmp, bytes, g->hlow_col, g->hpend[0], (unsigned)EL,
                                                                (unsigned)H, g->hlow_rp, g->hlow_rp + 1, 0, kbits, s);
        const hipError_t se = hipStreamSynchronize(s);
        gc_dfree(tmp);
        GC_HIP(e);
        GC_HIP(se);
        std::swap(g->hlow_col, g->hpend[0]);  // the unsorted copy becomes working memory
    }
    GC_HIP(hipMemsetAsync(pos, 0, sizeof(long long) * (size_t)(H + 1), s));
    pc.mark("hlow sort", s);
    hipLaunchKernelGGL(k_hch_count, dim3(grid_of(H + 1)), dim3(GC_BLOCK), 0, s, g->hlow_rp, H, pos);
    GC_HIP(gc_dmalloc((void**)&g->hch_rp, sizeof(long long) * (size_t)(H + 1)));
    if ((rc = scan_ll(pos, g->hch_rp, H + 1, s))) { gc_dfree(pos); return rc; }
    GC_READ(s, &g->nhch, (const long long*)g->hch_rp + H, 1);
    GC_HIP(gc_dmalloc((void**)&g->hch_own, sizeof(int) * (size_t)std::max<long long>(g->nhch, 1)));
    GC_HIP(gc_dmalloc((void**)&g->hkcnt, sizeof(int) * (size_t)H));
    GC_HIP(gc_dmalloc((void**)&g->hk, sizeof(unsigned) * (size_t)H));
    hipLaunchKernelGGL(k_hch_fill, dim3(grid_of(H)), dim3(GC_BLOCK), 0, s, g->hch_rp, H, g->hch_own);
    GC_HIP(hipGetLastError());
    GC_HIP(hipStreamSynchronize(s));
    gc_dfree(pos);
    g->hub_t = T;
    g->hub_w = W;
    pc.mark("chunks", s);
    if (pc.on) fprintf(stderr, "[gc hubs] H=%lld E=%lld EL=%lld\n", H, E, EL);
    return GC_OK;
}

}  // namespace

void gc_hubs_free(gc_graph* g) {
    void* ptrs[] = {g->hubpre, g->hperm, g->hid, g->hub_v, g->hin_rp, g->hin_col, g->hbits, g->hkill, g->hlow_rp, g->hlow_col,
                    g->hcur, g->hpc, g->hpend[0], g->hpend[1], g->hlow2[0], g->hlow2[1], g->hrow, g->hlen,
                    g->hch_rp, g->hch_own, g->hkcnt, g->hk, g->hcore, g->core_hub, g->core_bits, g->core_wcnt};
    for (void* p : ptrs)
        if (p) gc_dfree(p);
    gc_hub_bits_free(g);
    g->hubpre = nullptr;
    g->hperm = nullptr;
    g->hid = g->hub_v = g->hin_col = g->hlow_col = g->hcur = g->hpc = g->hpend[0] = g->hpend[1] = nullptr;
    g->hlow2[0] = g->hlow2[1] = g->hrow = g->hlen = nullptr;
    g->hin_rp = g->hlow_rp = g->hch_rp = nullptr;
    g->hch_own = g->hkcnt = nullptr;
    g->hk = nullptr;
    g->hcore = g->core_hub = nullptr;
    g->core_bits = nullptr;
    g->core_wcnt = nullptr;
    g->core_cap = 0;
    g->nhch = 0;
    g->hbits = g->hkill = nullptr;
    g->nhub = 0;
    g->hub_t = -1;
}

int gc_hub_threshold() { return env_int("GC_HUB_T", GC_HUB_T); }

int gc_hubs_prepare(gc_graph* g, GDev& d) {
    const int T = gc_hub_threshold();
    const int W = std::max(1, env_int("GC_HUB_W", GC_HUB_W));
    if (T < 0 || g->maxdeg <= T || g->borrowed) return GC_OK;
    // (hlow, the lower-rank hubs of each hub, follows the row partition it was built under)
    const bool stale = g->nhub && (g->hub_prio != g->part_prio || g->hub_seed != g->part_seed);
    if (g->hub_t != T || (g->nhub && g->hub_w != W) || stale) {
        gc_hubs_free(g);
        int rc = build(g, T, W);
        if (rc) {
            gc_hubs_free(g);
            return rc;
        }
    }
    g->hub_prio = g->part_prio;
    g->hub_seed = g->part_seed;
    if (g->nhub == 0) return GC_OK;
    GC_HIP(hipMemsetAsync(g->hbits, 0, sizeof(unsigned) * (size_t)g->nhub * g->hub_w, g->stream));
    d.heavy_t = T;
    d.hub_w = g->hub_w;
    d.hbits_w = g->hub_w;
    d.hid = g->hid;
    d.hub_v = g->hub_v;
    d.hin_rp = g->hin_rp;
    d.hin_col = g->hin_col;
    d.hbits = g->hbits;
    d.hb_stride = g->nhub;
    d.hkill = g->hkill;
    d.hlow_rp = g->hlow_rp;
    d.hlow_col = g->hlow_col;
    d.hcur = g->hcur;
    d.hpc = g->hpc;
    d.hpend[0] = g->hpend[0];
    d.hpend[1] = g->hpend[1];
    d.hrow = g->hrow;
    d.hlen = g->hlen;
    d.hlowb[0] = g->hlow_col;
    d.hlowb[1] = g->hlow2[0];
    d.hlowb[2] = g->hlow2[1];
    d.hub_long = env_int("GC_HUB_LONG", GC_HUB_LONG);
    d.tail_hmax = std::max(0, env_int("GC_TAIL_HMAX_HUB", GC_TAIL_HMAX_HUB));
    d.hch_rp = g->hch_rp;
    d.hch_own = g->hch_own;
    d.hkcnt = g->hkcnt;
    d.hk = g->hk;
    d.nhch = g->nhch;
    d.hub_scan = env_int("GC_HUB_SCAN", 1) > 0;
    d.hprep = !d.hub_scan && env_int("GC_HUB_PREP", 1) > 0 && g->nhch > 0 && d.hub_long >= 0;
    long long m = std::max<long long>(1, (long long)(0.6180339887 * (double)g->nhch));
    while (std::gcd(m, std::max<long long>(g->nhch, 1ll)) != 1) ++m;
    d.hch_mul = m;
    GC_HIP(hipMemsetAsync(g->hrow, 0, sizeof(int) * (size_t)g->nhub, g->stream));  // full rows again
    GC_HIP(hipMemsetAsync(g->hlen, 0, sizeof(int) * (size_t)g->nhub, g->stream));  // scan: no coloured prefix yet
    return GC_OK;
}

