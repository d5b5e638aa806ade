// gc_prep.hip -- the per-graph passes over every adjacency entry, edge-balanced:
//   * the rank partition of every row (the (deg, pos) order of coloring.py:64: lower-rank
//     neighbours first, so the Jones-Plassmann sweeps read only those),
//   * validate_graph_coloring's counts (coloring.py:149-162),
//   * the hub transpose of a symmetric graph (gc_hubs.hip: the hubs each row lists).
// All three are HBM/L2-bound integer gather work (one coalesced read of col, one random
// gather per entry, at most one coalesced write): no MFMA.
//
// Tiling.  The rows of R-MAT are power-law: a wave per 64 rows (round 2's kernels) walked
// the 4e5-entry hub rows serially and set the time of the whole pass (rank partition
// 133 + 99 ms, validation 65 ms on R-MAT-24).  Here the CSR is cut by merge path: tile t
// holds the rows whose key rp[r] + r falls in [t*GC_TW, (t+1)*GC_TW) -- at most GC_TW
// rows and, rows longer than GC_TH excepted, at most GC_TW + GC_TH entries, i.e. 16 per
// thread of a 256-thread workgroup.  A row longer than GC_TH (at most one per tile, its
// last) is cut into GC_SEG-entry segments handled like tiles; a pass that needs a row's
// prefix across its segments runs in two launches (counts, then positions).  The tiling
// depends on rp only: built once per graph.
//
// Within a tile the entries are staged in LDS with coalesced loads; thread t takes entries
// [16t, 16t + 16), finds its first row by binary search over the tile's row offsets (LDS)
// and walks on; its 16 gathers are issued together.  Per-row results come from ONE block
// scan of packed per-thread counts: a row's prefix at its start (recorded by the thread
// holding that start) and at its end give its counts and every entry's rank.
#include <cstring>

#include <rocprim/rocprim.hpp>

#include <algorithm>

#include "gc_device.h"
#include "gc_engine.h"

// GC_TILE_PER (build knob, default 8 since round 4): entries per thread.  The tile's LDS
// (~57 KB at 16) allowed two workgroups per CU; 8 halves it: R-MAT-24's step 171.2-173.5 ->
// 165.5-167.1 ms in an alternating A/B of the two builds (profiles/r04/c; A/B variant tile16)
#ifndef GC_TILE_PER
#define GC_TILE_PER 8
#endif
#define GC_PER GC_TILE_PER               // entries per thread: 256 x GC_PER = GC_TW + GC_TH = GC_SEG
#define GC_TW (GC_BLOCK / 2 * GC_PER)    // merge-path keys (rows + entries) per tile (2048 at 16)
#define GC_TH (GC_BLOCK / 2 * GC_PER)    // rows longer than this are split into segments
#define GC_SEG (GC_BLOCK * GC_PER)       // entries per segment (4096 at 16)
#define GC_PREP_GRID 4096

static_assert(GC_BLOCK * GC_PER == GC_TW + GC_TH && GC_BLOCK * GC_PER == GC_SEG, "tile geometry");
static_assert(GC_PER <= 16, "2-bit classes of a thread's entries are packed in one 32-bit word");

namespace {

// ------------------------------------------------------------------------------------
// tiling
// ------------------------------------------------------------------------------------
__global__ void k_tile_bounds(const long long* rp, long long n, long long ntiles, int* r0) {
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t <= ntiles;
         t += (long long)gridDim.x * blockDim.x) {
        if (t == ntiles) { r0[t] = (int)n; continue; }
        const long long target = t * GC_TW;
        long long lo = 0, hi = n;  // first r with rp[r] + r >= target (n if none)
        while (lo < hi) {
            const long long mid = (lo + hi) >> 1;
            if (rp[mid] + mid < target) lo = mid + 1;
            else hi = mid;
        }
        r0[t] = (int)lo;
    }
}

__global__ void k_tile_nseg(const long long* rp, const int* r0, long long ntiles, long long* cnt) {
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t <= ntiles;
         t += (long long)gridDim.x * blockDim.x) {
        long long c = 0;
        if (t < ntiles) {
            const int a = r0[t], b = r0[t + 1];
            if (b > a) {
                const long long d = rp[b] - rp[b - 1];
                if (d > GC_TH) c = (d + GC_SEG - 1) / GC_SEG;
            }
        }
        cnt[t] = c;
    }
}

__global__ void k_tile_segs(const int* r0, long long ntiles, const long long* base, int* seg_row, int* seg_j) {
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < ntiles;
         t += (long long)gridDim.x * blockDim.x) {
        const long long b0 = base[t], b1 = base[t + 1];
        if (b1 > b0) {
            const int v = r0[t + 1] - 1;
            for (long long j = 0; j < b1 - b0; ++j) {
                seg_row[b0 + j] = v;
                seg_j[b0 + j] = (int)j;
            }
        }
    }
}

struct Tiles {
    const long long* rp;
    const int* r0;
    long long ntiles;
    const long long* seg_base;  // [ntiles] = segment count
    const int* seg_row;
    const int* seg_j;
    int n;
};

__device__ __forceinline__ long long nseg_of(const Tiles& T) { return T.seg_base[T.ntiles]; }

// ------------------------------------------------------------------------------------
// block helpers
// ------------------------------------------------------------------------------------
// exclusive scan of a packed 64-bit count over the workgroup; *total = the sum
__device__ __forceinline__ ull block_excl_scan(ull x, ull* s_w, ull* total) {
    const int lane = gc_lane(), w = threadIdx.x / GC_WAVE;
    ull incl = x;
#pragma unroll
    for (int o = 1; o < GC_WAVE; o <<= 1) {
        const ull y = __shfl_up(incl, o, GC_WAVE);
        if (lane >= o) incl += y;
    }
    if (lane == GC_WAVE - 1) s_w[w] = incl;
    __syncthreads();
    ull pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < GC_WAVES_PER_BLOCK; ++i) {
        pre += i < w ? s_w[i] : 0ull;
        tot += s_w[i];
    }
    *total = tot;
    __syncthreads();
    return pre + incl - x;
}

__device__ __forceinline__ ull block_sum(ull x, ull* s_w) {
    ull t;
    block_excl_scan(x, s_w, &t);
    return t;
}

// packed class counts: 16 bits per class (a tile or segment holds <= 4096 entries)
__device__ __forceinline__ unsigned f16(ull p, int c) { return (unsigned)((p >> (16 * c)) & 0xFFFFull); }
__device__ __forceinline__ ull pack3(unsigned a, unsigned b, unsigned c) {
    return (ull)a | ((ull)b << 16) | ((ull)c << 32);
}
__device__ __forceinline__ ull pack4(unsigned a, unsigned b, unsigned c, unsigned d) {
    return pack3(a, b, c) | ((ull)d << 48);
}
// counts of this thread's entries [0, x) per class, from its 16-bit class masks
__device__ __forceinline__ ull own_before(unsigned m0, unsigned m1, unsigned m2, int x, unsigned m3 = 0u) {
    const unsigned lt = x >= 32 ? 0xFFFFFFFFu : ((1u << x) - 1u);
    return pack4(__popc(m0 & lt), __popc(m1 & lt), __popc(m2 & lt), __popc(m3 & lt));
}

// Tile rows into LDS: offsets relative to the first entry; returns R (rows) and sets *e_beg,
// *NE (light entries: the last row excluded when it is heavy), *heavy_last.
struct TileLds {
    int off[GC_TW + 1];
    unsigned key[GC_TW];     // per-row word of the pass (owner key / colour / nlow)
    int aux[GC_TW];          // second per-row word (hub index)
    ull base[GC_TW + 1];     // packed prefix at each row's start
    int buf[GC_TW + GC_TH];  // staged entries, then the pass's output
    ull w[GC_WAVES_PER_BLOCK];
    ull misc[4];
};
// GC_TILE_LDS_TRIM (build knob, default 1): each pass declares only the LDS rows it uses --
// the rank partition and the hub fill no `aux` (48 KB: three workgroups per CU where their
// registers allow, instead of two at 57 KB), the validation no `aux` / `base` (32 KB: four,
// its register limit).  The tiles are latency-bound chains (~4 dependent memory trips each),
// so more resident workgroups are more tiles in flight.  0: every pass the full TileLds.
#ifndef GC_TILE_LDS_TRIM
#define GC_TILE_LDS_TRIM 1
#endif
#if GC_TILE_LDS_TRIM
struct TileLdsP {  // rank partition, hub fill
    int off[GC_TW + 1];
    unsigned key[GC_TW];
    ull base[GC_TW + 1];
    int buf[GC_TW + GC_TH];
    ull w[GC_WAVES_PER_BLOCK];
    ull misc[4];
};
struct TileLdsV {  // validation
    int off[GC_TW + 1];
    unsigned key[GC_TW];
    int nl[GC_TW];
    int buf[GC_TW + GC_TH];
    ull w[GC_WAVES_PER_BLOCK];
    ull misc[4];
};
#else
typedef TileLds TileLdsP;
typedef TileLds TileLdsV;
#endif

template <class Lds>
__device__ __forceinline__ int tile_rows(const Tiles& T, long long t, Lds& S, int* r0o, long long* e_beg, int* NE,
                                         bool* heavy_last) {
    const int r0 = T.r0[t], r1 = T.r0[t + 1];
    const int R = r1 - r0;
    *r0o = r0;
    if (R == 0) return 0;
    const long long eb = T.rp[r0];
    for (int i = threadIdx.x; i <= R; i += blockDim.x) S.off[i] = (int)(T.rp[r0 + i] - eb);
    __syncthreads();
    const bool hl = S.off[R] - S.off[R - 1] > GC_TH;
    *e_beg = eb;
    *NE = hl ? S.off[R - 1] : S.off[R];
    *heavy_last = hl;
    return R;
}

// this thread's entries [j0, j0 + nv) of the staged tile, with their rows
template <class Lds>
__device__ __forceinline__ int thread_entries(const Lds& S, int R, int NE, int* u, int* rk) {
    const int j0 = threadIdx.x * GC_PER;
    int nv = NE - j0;
    nv = nv < 0 ? 0 : (nv > GC_PER ? GC_PER : nv);
    if (nv == 0) return 0;
    int lo = 0, hi = R - 1;  // last r with off[r] <= j0
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (S.off[mid] <= j0) lo = mid;
        else hi = mid - 1;
    }
    int r = lo;
#pragma unroll
    for (int k = 0; k < GC_PER; ++k) {
        if (k < nv) {
            const int j = j0 + k;
            while (S.off[r + 1] <= j) ++r;
            rk[k] = r;
            u[k] = S.buf[j];
        } else {
            rk[k] = 0;
            u[k] = 0;
        }
    }
    return nv;
}

// Row bases: the thread holding a row's first entry records prefix + its own entries before
// it; rows starting at or past NE get the total.  Then base[R] = total.
template <class Lds>
__device__ __forceinline__ void record_bases(Lds& S, int R, int NE, int nv, ull prefix, ull total, unsigned m0,
                                             unsigned m1, unsigned m2, unsigned m3 = 0u) {
    const int j0 = threadIdx.x * GC_PER;
    if (nv > 0) {
        int lo = 0, hi = R;  // first r with off[r] >= j0
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (S.off[mid] < j0) lo = mid + 1;
            else hi = mid;
        }
        for (int r = lo; r < R && S.off[r] < j0 + nv; ++r) S.base[r] = prefix + own_before(m0, m1, m2, S.off[r] - j0, m3);
    }
    for (int r = threadIdx.x; r <= R; r += blockDim.x)
        if (S.off[r] >= NE) S.base[r] = total;
}

// ------------------------------------------------------------------------------------
// rank partition
// ------------------------------------------------------------------------------------
struct PartArgs {
    Tiles T;
    const int* src;
    int* dst;
    const int* deg;
    const unsigned char* kb;
    int* nlow;
    int* neq;
    int* nhe;
    ull seed;
    ull* bad;
    ull* seg_aux;       // per segment: packed class counts
    unsigned* seg_cls;  // per segment x thread: 2-bit classes (bits 0..15), hub flags (bits 16..23)
    unsigned char* hflag;  // or null: byte per output entry, 1 iff the entry is a hub (deg > hub_t)
    int hub_t;
    unsigned hub_code;  // gc_deg_code(hub_t + 1)
    int hub_amb;        // the code's bucket also holds degrees <= hub_t: those entries gather deg
};

// Hub flags need a third bit per entry in seg_cls (8 entries per thread: bits 16..23).
#define GC_PART_HUBFLAG (GC_PER <= 8)

__device__ __forceinline__ unsigned owner_key(const PartArgs& a, int prio, int v) {
    return prio ? gc_prio_hash(a.seed, v) : (unsigned)a.deg[v];
}

// classes of this thread's entries against their owners' keys: 0 lower key, 1 equal key and
// earlier position, 2 higher key and earlier position, 3 the rest (equal key and later
// position, higher key and later position, self-loops, out-of-range entries).  Classes 1 + 2
// are the entries an arrival of the owner can be refused by in variant B's fold (earlier,
// degree >= its own), class 3 holds the ones it can be evicted by (later, higher degree).
// The seeded-priority partition (PRIO) has classes 0 and 3 only.
template <int PRIO>
__device__ __forceinline__ void classify(const PartArgs& a, int nv, const int* u, const unsigned* kv, const int* v,
                                         unsigned* m0, unsigned* m1, unsigned* m2, unsigned* m3, ull* nbad,
                                         unsigned* mh) {
    // the class masks are built directly (no per-entry class array: registers, occupancy)
    unsigned a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    *mh = 0;
    if (PRIO) {
#pragma unroll
        for (int k = 0; k < GC_PER; ++k) {
            if (k < nv) {
                const unsigned bit = 1u << k;
                if ((unsigned)u[k] >= (unsigned)a.T.n) { a3 |= bit; ++*nbad; continue; }
                const unsigned ku = gc_prio_hash(a.seed, u[k]);
                if (gc_rank_lt_key(ku, u[k], kv[k], v[k])) a0 |= bit;
                else a3 |= bit;
            }
        }
    } else {
        // the byte key first (gc_deg_code: 16.8 MB against 67 MB of deg on R-MAT-24), the
        // full degree only when both codes are equal and bucketed (>= GC_DEG_CODE_EXACT)
        unsigned kb8[GC_PER];
#pragma unroll
        for (int k = 0; k < GC_PER; ++k) {
            const bool ok = k < nv && (unsigned)u[k] < (unsigned)a.T.n;
            kb8[k] = ok ? (unsigned)a.kb[u[k]] : 0u;
        }
        // fullm: entries whose class needs the full degree (equal bucketed codes); hamb: entries
        // whose hub flag does (the key's bucket straddles the hub threshold) -- one gather pass
        // serves both, and bit masks keep the registers of the flag-free kernel (occupancy)
        unsigned fullm = 0, hamb = 0, h = 0;
        const unsigned hc = a.hub_code;
        const bool hf = a.hflag != nullptr;
#pragma unroll
        for (int k = 0; k < GC_PER; ++k) {
            if (k < nv) {
                const unsigned bit = 1u << k;
                if ((unsigned)u[k] >= (unsigned)a.T.n) { a3 |= bit; ++*nbad; continue; }
                const unsigned kv8 = gc_deg_code((long long)kv[k]);
                const bool early = u[k] < v[k];
                if (kb8[k] != kv8) {
                    if (kb8[k] < kv8) a0 |= bit;
                    else if (early) a2 |= bit;
                    else a3 |= bit;
                } else if (kv8 < GC_DEG_CODE_EXACT) {
                    if (early) a1 |= bit;
                    else a3 |= bit;
                } else {
                    fullm |= bit;
                }
                // hub entries (deg(u) > hub_t) from the same byte key: exact except in the
                // code's bucket when it also holds degrees <= hub_t (R-MAT: few entries)
                if (hf && kb8[k] >= hc) {
                    if (kb8[k] > hc || !a.hub_amb) h |= bit;
                    else hamb |= bit;
                }
            }
        }
        if (fullm | hamb) {
            unsigned du[GC_PER];
#pragma unroll
            for (int k = 0; k < GC_PER; ++k) du[k] = ((fullm | hamb) >> k) & 1u ? (unsigned)a.deg[u[k]] : 0u;
#pragma unroll
            for (int k = 0; k < GC_PER; ++k) {
                const unsigned bit = 1u << k;
                if (fullm & bit) {
                    if (du[k] < kv[k]) a0 |= bit;
                    else if (u[k] >= v[k]) a3 |= bit;
                    else if (du[k] > kv[k]) a2 |= bit;
                    else a1 |= bit;
                }
                if ((hamb & bit) && du[k] > (unsigned)a.hub_t) h |= bit;
            }
        }
        *mh = h;
    }
    *m0 = a0;
    *m1 = a1;
    *m2 = a2;
    *m3 = a3;
}

template <int PRIO>
__device__ void part_tile(const PartArgs& a, TileLdsP& S, long long t, ull* nbad) {
    int r0, NE;
    long long eb;
    bool hl;
    const int R = tile_rows(a.T, t, S, &r0, &eb, &NE, &hl);
    if (R == 0) return;
    for (int i = threadIdx.x; i < R; i += blockDim.x) S.key[i] = owner_key(a, PRIO, r0 + i);
    for (int i = threadIdx.x; i < NE; i += blockDim.x) S.buf[i] = a.src[eb + i];
    __syncthreads();
    int u[GC_PER], rk[GC_PER];
    const int nv = thread_entries(S, R, NE, u, rk);
    unsigned kv[GC_PER];
    int vv[GC_PER];
#pragma unroll
    for (int k = 0; k < GC_PER; ++k) {
        kv[k] = S.key[rk[k]];
        vv[k] = r0 + rk[k];
    }
    unsigned m0, m1, m2, m3, mh;
    classify<PRIO>(a, nv, u, kv, vv, &m0, &m1, &m2, &m3, nbad, &mh);
    const ull mine = pack4(__popc(m0), __popc(m1), __popc(m2), __popc(m3));
    ull total;
    const ull prefix = block_excl_scan(mine, S.w, &total);  // (its barriers: every S.buf read is done)
    record_bases(S, R, NE, nv, prefix, total, m0, m1, m2, m3);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < GC_PER; ++k) {
        if (k >= nv) break;
        const int r = rk[k];
        const ull b = S.base[r], b1 = S.base[r + 1];
        const unsigned c0 = f16(b1, 0) - f16(b, 0), c1 = f16(b1, 1) - f16(b, 1), c2 = f16(b1, 2) - f16(b, 2);
        const unsigned bit = 1u << k;
        const int c = (m0 & bit) ? 0 : ((m1 & bit) ? 1 : ((m2 & bit) ? 2 : 3));
        const unsigned mc = c == 0 ? m0 : (c == 1 ? m1 : (c == 2 ? m2 : m3));
        const unsigned rank = f16(prefix, c) + __popc(mc & (bit - 1u)) - f16(b, c);
        const unsigned start = c == 0 ? 0u : (c == 1 ? c0 : (c == 2 ? c0 + c1 : c0 + c1 + c2));
        // (a hub entry carries its flag in bit 31: vertex ids are < 2^31)
        S.buf[S.off[r] + (int)(start + rank)] = (int)((unsigned)u[k] | (((mh >> k) & 1u) << 31));
    }
    __syncthreads();
    if (a.hflag) {
        for (int i = threadIdx.x; i < NE; i += blockDim.x) {
            const unsigned x = (unsigned)S.buf[i];
            a.dst[eb + i] = (int)(x & 0x7FFFFFFFu);
            a.hflag[eb + i] = (unsigned char)(x >> 31);
        }
    } else {
        for (int i = threadIdx.x; i < NE; i += blockDim.x) a.dst[eb + i] = S.buf[i];
    }
    for (int r = threadIdx.x; r < R; r += blockDim.x) {
        if (hl && r == R - 1) continue;  // the heavy row: its segments' second pass
        const ull b = S.base[r], b1 = S.base[r + 1];
        const unsigned c0 = f16(b1, 0) - f16(b, 0), c1 = f16(b1, 1) - f16(b, 1);
        a.nlow[r0 + r] = (int)(c0 + c1);
        if (a.neq) a.neq[r0 + r] = (int)c1;
        if (a.nhe) a.nhe[r0 + r] = (int)(f16(b1, 2) - f16(b, 2));
    }
}

// segment of a heavy row, first pass: classes (kept for the second pass) and counts
template <int PRIO>
__device__ void part_seg1(const PartArgs& a, TileLdsP& S, long long s, ull* nbad) {
    const int v = a.T.seg_row[s], j = a.T.seg_j[s];
    const long long rs = a.T.rp[v], d = a.T.rp[v + 1] - rs;
    const long long e0 = rs + (long long)j * GC_SEG;
    const int len = (int)std::min<long long>(GC_SEG, d - (long long)j * GC_SEG);
    const unsigned key = owner_key(a, PRIO, v);
    for (int i = threadIdx.x; i < len; i += blockDim.x) S.buf[i] = a.src[e0 + i];
    __syncthreads();
    const int j0 = threadIdx.x * GC_PER;
    int nv = len - j0;
    nv = nv < 0 ? 0 : (nv > GC_PER ? GC_PER : nv);
    int u[GC_PER], vv[GC_PER];
    unsigned kv[GC_PER];
#pragma unroll
    for (int k = 0; k < GC_PER; ++k) {
        u[k] = k < nv ? S.buf[j0 + k] : 0;
        vv[k] = v;
        kv[k] = key;
    }
    unsigned m0, m1, m2, m3, mh;
    classify<PRIO>(a, nv, u, kv, vv, &m0, &m1, &m2, &m3, nbad, &mh);
    unsigned cls = 0;  // 2 bits per entry: its class
#pragma unroll
    for (int k = 0; k < GC_PER; ++k)
        cls |= (((m1 >> k) & 1u) | (((m2 >> k) & 1u) << 1) | (((m3 >> k) & 1u) * 3u)) << (2 * k);
#if GC_PART_HUBFLAG
    cls |= mh << 16;
#endif
    a.seg_cls[s * GC_BLOCK + threadIdx.x] = cls;
    const ull tot = block_sum(pack4(__popc(m0), __popc(m1), __popc(m2), __popc(m3)), S.w);
    if (threadIdx.x == 0) a.seg_aux[s] = tot;
}

template <int PRIO>
__global__ void __launch_bounds__(GC_BLOCK) k_part1(PartArgs a) {
    __shared__ TileLdsP S;
    const long long nt = a.T.ntiles, ns = nseg_of(a.T);
    ull nbad = 0;
    for (long long it = blockIdx.x; it < nt + ns; it += gridDim.x) {
        if (it < nt) part_tile<PRIO>(a, S, it, &nbad);
        else part_seg1<PRIO>(a, S, it - nt, &nbad);
        __syncthreads();
    }
    nbad = gc_wave_sum(nbad);
    if (gc_lane() == 0 && nbad) atomicAdd(a.bad, nbad);
}

// sums over segments [f, l) of a row's packed counts, per class (one wave, lane-strided)
__device__ __forceinline__ void seg_sums(const ull* aux, long long f, long long l, ull* c) {
    ull a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    for (long long i = f + gc_lane(); i < l; i += GC_WAVE) {
        const ull p = aux[i];
        a0 += f16(p, 0);
        a1 += f16(p, 1);
        a2 += f16(p, 2);
        a3 += f16(p, 3);
    }
    c[0] = gc_wave_sum(a0);
    c[1] = gc_wave_sum(a1);
    c[2] = gc_wave_sum(a2);
    c[3] = gc_wave_sum(a3);
}

// second pass of the heavy rows: every segment places its entries after the row's earlier
// segments' entries of the same class
__global__ void __launch_bounds__(GC_BLOCK) k_part2(PartArgs a) {
    __shared__ int buf[GC_SEG];
    __shared__ ull s_w[GC_WAVES_PER_BLOCK];
    __shared__ ull s_pre[4], s_tot[4];
    const long long ns = nseg_of(a.T);
    for (long long s = blockIdx.x; s < ns; s += gridDim.x) {
        const int v = a.T.seg_row[s], j = a.T.seg_j[s];
        const long long rs = a.T.rp[v], d = a.T.rp[v + 1] - rs;
        const long long e0 = rs + (long long)j * GC_SEG;
        const int len = (int)std::min<long long>(GC_SEG, d - (long long)j * GC_SEG);
        const long long first = s - j, nsr = (d + GC_SEG - 1) / GC_SEG;
        if (threadIdx.x < GC_WAVE) {
            ull p[4], t[4];
            seg_sums(a.seg_aux, first, s, p);
            seg_sums(a.seg_aux, first, first + nsr, t);
            if (threadIdx.x == 0)
                for (int c = 0; c < 4; ++c) {
                    s_pre[c] = p[c];
                    s_tot[c] = t[c];
                }
        }
        for (int i = threadIdx.x; i < len; i += blockDim.x) buf[i] = a.src[e0 + i];
        __syncthreads();
        const int j0 = threadIdx.x * GC_PER;
        int nv = len - j0;
        nv = nv < 0 ? 0 : (nv > GC_PER ? GC_PER : nv);
        const unsigned cls = a.seg_cls[s * GC_BLOCK + threadIdx.x];
#if GC_PART_HUBFLAG
        const unsigned mh = a.hflag ? cls >> 16 : 0u;
#else
        const unsigned mh = 0u;
#endif
        int u[GC_PER];
        unsigned m0 = 0, m1 = 0, m2 = 0, m3 = 0;
#pragma unroll
        for (int k = 0; k < GC_PER; ++k) {
            u[k] = k < nv ? buf[j0 + k] : 0;
            if (k < nv) {
                const unsigned c = (cls >> (2 * k)) & 3u;
                m0 |= (c == 0 ? 1u : 0u) << k;
                m1 |= (c == 1 ? 1u : 0u) << k;
                m2 |= (c == 2 ? 1u : 0u) << k;
                m3 |= (c == 3 ? 1u : 0u) << k;
            }
        }
        ull segtot;
        const ull prefix = block_excl_scan(pack4(__popc(m0), __popc(m1), __popc(m2), __popc(m3)), s_w, &segtot);
        const unsigned L0 = f16(segtot, 0), L1 = f16(segtot, 1), L2 = f16(segtot, 2);
        // compact the segment in LDS by class (u is in registers; block_excl_scan's barriers
        // ordered every read of buf before these writes)
#pragma unroll
        for (int k = 0; k < GC_PER; ++k) {
            if (k >= nv) break;
            const unsigned bit = 1u << k;
            const int c = (m0 & bit) ? 0 : ((m1 & bit) ? 1 : ((m2 & bit) ? 2 : 3));
            const unsigned mc = c == 0 ? m0 : (c == 1 ? m1 : (c == 2 ? m2 : m3));
            const unsigned sec = c == 0 ? 0u : (c == 1 ? L0 : (c == 2 ? L0 + L1 : L0 + L1 + L2));
            buf[sec + f16(prefix, c) + __popc(mc & (bit - 1u))] = (int)((unsigned)u[k] | (((mh >> k) & 1u) << 31));
        }
        __syncthreads();
        const long long T0 = (long long)s_tot[0], T1 = (long long)s_tot[1], T2 = (long long)s_tot[2];
        const long long P0 = (long long)s_pre[0], P1 = (long long)s_pre[1], P2 = (long long)s_pre[2],
                        P3 = (long long)s_pre[3];
        for (int i = threadIdx.x; i < len; i += blockDim.x) {
            long long pos;
            if (i < (int)L0) pos = P0 + i;
            else if (i < (int)(L0 + L1)) pos = T0 + P1 + (i - (int)L0);
            else if (i < (int)(L0 + L1 + L2)) pos = T0 + T1 + P2 + (i - (int)(L0 + L1));
            else pos = T0 + T1 + T2 + P3 + (i - (int)(L0 + L1 + L2));
            const unsigned x = (unsigned)buf[i];
            if (a.hflag) {
                a.dst[rs + pos] = (int)(x & 0x7FFFFFFFu);
                a.hflag[rs + pos] = (unsigned char)(x >> 31);
            } else {
                a.dst[rs + pos] = (int)x;
            }
        }
        if (j == 0 && threadIdx.x == 0) {
            a.nlow[v] = (int)(T0 + T1);
            if (a.neq) a.neq[v] = (int)T1;
            if (a.nhe) a.nhe[v] = (int)T2;
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------
// validate_graph_coloring counts (coloring.py:149-162): #(colour == -1) over the vertices,
// #{(v, u): u listed in N(v), colour[u] == colour[v]} over the entries (directed, duplicates
// and self-loops count, exactly as coloring.py:157-158)
// ------------------------------------------------------------------------------------
// C8 (GC_VALIDATE_C8=1, staged in round 3; the resident colouring only): the neighbours'
// colours are gathered from the byte mirror c8 (n bytes instead of 4n: R-MAT-26 67 MB against
// 268 MB of random-gather footprint), the int colour only when both bytes say ">= 254".
// Colour equality == equal bytes and (byte < 254 or equal ints), since c8 = gc_c8_of(colour).
__device__ __forceinline__ bool same_colour8(const int* colors, int u, unsigned cu8, int cv) {
    const unsigned cv8 = gc_c8_of(cv);
    return cu8 == cv8 && (cv8 != GC_C8_BIG || colors[u] == cv);
}
// HALF (round 4; symmetric graphs): an entry (v, u), u != v, and its mirror (u, v) are one
// conflict each or neither, and exactly one of them lies in a low part (the rank partition:
// lower rank first; a strict order, so a self-loop is never low).  So the directed count is
// 2 x the conflicts of the low parts + the self-loop entries (a self-loop always conflicts),
// and only the low entries are gathered: half the gathers, col still read whole (the rows
// are staged tile by tile).  Duplicates mirror too: each copy counts on both sides.

// Rows [V.lo, V.hi) only (gc_validate_range): the tiles [t0, t1) and segments [s0, s1) that
// hold them; rows of a boundary tile outside the range are skipped.
struct VRange {
    long long t0, t1, s0, s1;
    int lo, hi;
};

template <int C8, int HALF>
__global__ void __launch_bounds__(GC_BLOCK) k_validate_tiles(Tiles T, VRange V, const int* col, const int* colors,
                                                             const unsigned char* c8, const int* nlow, ull* unc_out,
                                                             ull* conf_out) {
    __shared__ TileLdsV S;
    const long long nt = V.t1 - V.t0, ns = V.s1 - V.s0;
    ull unc = 0, conf = 0;
    for (long long q = blockIdx.x; q < nt + ns; q += gridDim.x) {
        if (q < nt) {
            const long long it = V.t0 + q;
            int r0, NE;
            long long eb;
            bool hl;
            const int R = tile_rows(T, it, S, &r0, &eb, &NE, &hl);
            if (R == 0) continue;
            for (int i = threadIdx.x; i < R; i += blockDim.x) {
                const int cv = colors[r0 + i];
                S.key[i] = (unsigned)cv;
                if (HALF) S.nl[i] = nlow[r0 + i];
                unc += cv == -1 && r0 + i >= V.lo && r0 + i < V.hi;
            }
            for (int i = threadIdx.x; i < NE; i += blockDim.x) S.buf[i] = col[eb + i];
            __syncthreads();
            int u[GC_PER], rk[GC_PER];
            const int nv = thread_entries(S, R, NE, u, rk);
            bool on[GC_PER];  // entries whose colour is gathered
#pragma unroll
            for (int k = 0; k < GC_PER; ++k) {
                on[k] = k < nv && r0 + rk[k] >= V.lo && r0 + rk[k] < V.hi;
                if (HALF && on[k]) {
                    const int j = threadIdx.x * GC_PER + k;  // thread_entries' entry j0 + k
                    conf += u[k] == r0 + rk[k] ? 1 : 0;     // a self-loop
                    on[k] = j - S.off[rk[k]] < S.nl[rk[k]];
                }
            }
            int cu[GC_PER];
#pragma unroll
            for (int k = 0; k < GC_PER; ++k) cu[k] = on[k] ? (C8 ? (int)c8[u[k]] : colors[u[k]]) : 0;
            ull lc = 0;
            if (C8) {
#pragma unroll
                for (int k = 0; k < GC_PER; ++k)
                    lc += (on[k] && same_colour8(colors, u[k], (unsigned)cu[k], (int)S.key[rk[k]])) ? 1 : 0;
            } else {
#pragma unroll
                for (int k = 0; k < GC_PER; ++k) lc += (on[k] && cu[k] == (int)S.key[rk[k]]) ? 1 : 0;
            }
            conf += HALF ? 2 * lc : lc;
        } else {
            const long long s = V.s0 + (q - nt);
            const int v = T.seg_row[s], j = T.seg_j[s];
            if (v < V.lo || v >= V.hi) continue;  // (uniform per workgroup: no barrier skipped)
            const long long rs = T.rp[v], d = T.rp[v + 1] - rs;
            const long long e0 = rs + (long long)j * GC_SEG;
            const int len = (int)std::min<long long>(GC_SEG, d - (long long)j * GC_SEG);
            const int lowlen = HALF ? (int)std::max<long long>(0, std::min<long long>(len, nlow[v] - (long long)j * GC_SEG)) : len;
            const int cv = colors[v];
            int uu[GC_PER], cu[GC_PER];
#pragma unroll
            for (int k = 0; k < GC_PER; ++k) {  // coalesced: entry threadIdx + k * 256
                const int i = threadIdx.x + k * GC_BLOCK;
                uu[k] = i < len ? col[e0 + i] : 0;
                if (HALF) conf += (i < len && uu[k] == v) ? 1 : 0;  // a self-loop
            }
#pragma unroll
            for (int k = 0; k < GC_PER; ++k) {
                const int i = threadIdx.x + k * GC_BLOCK;
                cu[k] = i < lowlen ? (C8 ? (int)c8[uu[k]] : colors[uu[k]]) : 0;
            }
            ull lc = 0;
            if (C8) {
#pragma unroll
                for (int k = 0; k < GC_PER; ++k)
                    lc += (threadIdx.x + k * GC_BLOCK < lowlen && same_colour8(colors, uu[k], (unsigned)cu[k], cv)) ? 1 : 0;
            } else {
#pragma unroll
                for (int k = 0; k < GC_PER; ++k) lc += (threadIdx.x + k * GC_BLOCK < lowlen && cu[k] == cv) ? 1 : 0;
            }
            conf += HALF ? 2 * lc : lc;
        }
        __syncthreads();
    }
    unc = gc_wave_sum(unc);
    conf = gc_wave_sum(conf);
    if (gc_lane() == 0) {
        if (unc) atomicAdd(unc_out, unc);
        if (conf) atomicAdd(conf_out, conf);
    }
}

// ------------------------------------------------------------------------------------
// hub transpose of a symmetric graph: the rows that list hub x are x's own entries, so the
// hubs each row u lists (hin, pushed into by u's commits) are u's entries that are hubs --
// a filter of every row, no atomics on targets.  A hub row's lower-rank hubs (hlow) are the
// entries of its hin row that lie in its low part: a prefix of that row (klow of them).
//
// Round 4: a rank structure over the entries instead of edge-balanced tiles.  Bit e of
// `hb_bits` says whether entry e (col[e]) is a hub; `hb_wpre` is the exclusive prefix of the
// words' popcounts, so rank(e) = the hub entries before position e = wpre[e/64] +
// popc(bits[e/64] below e).  Then hin_rp[u] = rank(rp[u]) (rows in order, entries in row
// order: the same hin rows as a per-row filter), klow[x] = rank(rp[v] + nlow[v]) -
// rank(rp[v]) for hub v = hub_v[x], and entry e goes to hin_col[rank(e)].  Two coalesced
// streams over col (bits; fill) instead of two passes of LDS-staged tiles with a row search
// per thread (round 3: R-MAT-26 hin count 24 ms + fill 51 ms, ~0.04 of the HBM peak).
// Per entry: 4 B of col (both passes) + one hubmap gather (bits pass); per hub entry: 4 B
// written + the hub-index gathers (hubpre / hubmap / hperm: 2 x n/8 + 4 H bytes, L2/MALL).

// hubmap and hubpre interleaved per word (hb_mp, built for the transpose and freed after
// it): one 8-byte gather gives an entry's hub bit and its word's id-order base -- both
// passes are bound by their gather rate (~270 G/s on R-MAT-24), and the fill's per-hub-entry
// lookup is then two gathers (this word, hperm) instead of three
__global__ void k_hb_mp(const unsigned* hubmap, const unsigned* hubpre, long long words, uint2* mp) {
    for (long long w = (long long)blockIdx.x * blockDim.x + threadIdx.x; w < words; w += (long long)gridDim.x * blockDim.x)
        mp[w] = make_uint2(hubmap[w], hubpre[w]);
}

// bits of 64 consecutive words per wave and iteration; lane k keeps word w0 + k (coalesced
// stores), 8 entry loads per lane in flight
__global__ void __launch_bounds__(GC_BLOCK) k_hbit(const int* col, long long nnz, long long n, const uint2* mp,
                                                  ull* bits, long long* wcnt, long long nw) {
    const int lane = gc_lane();
    const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / GC_WAVE;
    const long long nwaves = (long long)gridDim.x * blockDim.x / GC_WAVE;
    for (long long w0 = wave * GC_WAVE; w0 < nw; w0 += nwaves * GC_WAVE) {
        ull mine = 0;
#pragma unroll 1
        for (int k0 = 0; k0 < GC_WAVE; k0 += 8) {
            int u[8];
            unsigned hw[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const long long e = (w0 + k0 + k) * GC_WAVE + lane;
                u[k] = e < nnz ? col[e] : -1;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) hw[k] = (u[k] >= 0 && (long long)u[k] < n) ? mp[u[k] >> 5].x : 0u;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const ull m = __ballot(u[k] >= 0 && ((hw[k] >> (u[k] & 31)) & 1u));
                if (lane == k0 + k) mine = m;
            }
        }
        const long long w = w0 + lane;
        if (w < nw) {
            bits[w] = mine;
            wcnt[w] = (long long)__popcll(mine);
        }
    }
}

// the same bits from the rank partition's hub flags (gc_graph::hubflag, a byte per entry):
// a coalesced byte stream per wave, no gather
__global__ void __launch_bounds__(GC_BLOCK) k_hbit_flags(const unsigned char* flag, long long nnz, ull* bits,
                                                        long long* wcnt, long long nw) {
    const int lane = gc_lane();
    const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / GC_WAVE;
    const long long nwaves = (long long)gridDim.x * blockDim.x / GC_WAVE;
    for (long long w0 = wave * GC_WAVE; w0 < nw; w0 += nwaves * GC_WAVE) {
        ull mine = 0;
#pragma unroll 1
        for (int k0 = 0; k0 < GC_WAVE; k0 += 8) {
            unsigned f[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const long long e = (w0 + k0 + k) * GC_WAVE + lane;
                f[k] = e < nnz ? (unsigned)flag[e] : 0u;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const ull m = __ballot(f[k] != 0u);
                if (lane == k0 + k) mine = m;
            }
        }
        const long long w = w0 + lane;
        if (w < nw) {
            bits[w] = mine;
            wcnt[w] = (long long)__popcll(mine);
        }
    }
}

__device__ __forceinline__ long long hb_rank(const ull* bits, const long long* wpre, long long e) {
    const long long w = e >> 6;
    const int b = (int)(e & 63);
    return wpre[w] + (long long)__popcll(bits[w] & ((1ull << b) - 1ull));
}

// hin_rp[u] = rank(rp[u]) for u in [0, n] (hin_rp[n] = E); klow of every hub row
__global__ void __launch_bounds__(GC_BLOCK) k_hin_rank(const long long* rp, long long n, const ull* bits,
                                                      const long long* wpre, const int* nlow, const int* hid,
                                                      long long* hin_rp, long long* klow) {
    for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v <= n; v += (long long)gridDim.x * blockDim.x) {
        const long long e = rp[v];
        const long long r = hb_rank(bits, wpre, e);
        hin_rp[v] = r;
        if (v < n) {
            const int x = hid[v];
            if (x >= 0) klow[x] = hb_rank(bits, wpre, e + nlow[v]) - r;
        }
    }
}

// hin_col[rank(e)] = hub index of col[e] for every hub entry e: a wave per 64 words, lane k
// holding word w0 + k's bits and prefix, 8 words' entries in flight per step
__global__ void __launch_bounds__(GC_BLOCK) k_hin_fill(const int* col, long long nw, const ull* bits,
                                                      const long long* wpre, const uint2* mp, const int* hperm,
                                                      int* hin_col) {
    const int lane = gc_lane();
    const ull lt = gc_lanemask_lt();
    const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / GC_WAVE;
    const long long nwaves = (long long)gridDim.x * blockDim.x / GC_WAVE;
    for (long long w0 = wave * GC_WAVE; w0 < nw; w0 += nwaves * GC_WAVE) {
        const ull myb = w0 + lane < nw ? bits[w0 + lane] : 0ull;
        const long long myp = w0 + lane < nw ? wpre[w0 + lane] : 0ll;
#pragma unroll 1
        for (int k0 = 0; k0 < GC_WAVE; k0 += 8) {
            ull mk[8];
            long long base[8];
            int u[8];
            bool on[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                mk[k] = __shfl(myb, k0 + k, GC_WAVE);
                base[k] = __shfl(myp, k0 + k, GC_WAVE);
                on[k] = (mk[k] >> lane) & 1ull;
                u[k] = on[k] ? col[(w0 + k0 + k) * GC_WAVE + lane] : 0;
            }
            uint2 m[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) m[k] = on[k] ? mp[u[k] >> 5] : make_uint2(0u, 0u);
            int x[8];
#pragma unroll
            for (int k = 0; k < 8; ++k)
                x[k] = on[k] ? hperm[m[k].y + __popc(m[k].x & ((1u << (u[k] & 31)) - 1u))] : 0;
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (on[k]) hin_col[base[k] + __popcll(mk[k] & lt)] = x[k];
        }
    }
}

// hlow rows: the klow-entry prefix of each hub's hin row (a wave per hub)
__global__ void k_hlow_copy(const int* hub_v, long long H, const long long* hin_rp, const int* hin_col,
                            const long long* hlow_rp, int* hlow_col) {
    const long long waves = (long long)gridDim.x * (blockDim.x / GC_WAVE);
    for (long long x = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / GC_WAVE; x < H; x += waves) {
        const long long src = hin_rp[hub_v[x]], dst = hlow_rp[x], len = hlow_rp[x + 1] - dst;
        for (long long i = gc_lane(); i < len; i += GC_WAVE) hlow_col[dst + i] = hin_col[src + i];
    }
}

int scan_ll(const long long* in, long long* out, long long count, hipStream_t s) {
    size_t bytes = 0;
    GC_HIP(rocprim::exclusive_scan(nullptr, bytes, in, out, 0ll, (size_t)count, rocprim::plus<long long>(), s));
    void* tmp = nullptr;
    GC_HIP(gc_dmalloc(&tmp, bytes ? bytes : 1));
    hipError_t e = rocprim::exclusive_scan(tmp, bytes, in, out, 0ll, (size_t)count, rocprim::plus<long long>(), s);
    const hipError_t se = hipStreamSynchronize(s);  // the temporary goes back to the cache idle
    gc_dfree(tmp);
    GC_HIP(e);
    GC_HIP(se);
    return GC_OK;
}

// ------------------------------------------------------------------------------------
// A shard's in-rows of a symmetric graph (gc_shard_create): for every row v, its entries in
// the shard's vertex range [lo, hi), in row order (trp / tcol).  Entry-parallel over the tiles
// and the heavy rows' segments, like the rank partition: round 4's wave-per-row kernels took
// 1.73 s on R-MAT-28 (a row per wave, the heaviest rows one wave each; profiles/r05/v).
// ------------------------------------------------------------------------------------
// pass 1: per-row counts (tiles: plain stores; heavy rows: per-segment counts, summed)
__global__ void __launch_bounds__(GC_BLOCK) k_filt_count(Tiles T, const int* col, int lo, int hi, long long* cnt,
                                                         ull* segc) {
    __shared__ TileLdsP S;
    const long long nt = T.ntiles, ns = nseg_of(T);
    for (long long q = blockIdx.x; q < nt + ns; q += gridDim.x) {
        if (q < nt) {
            int r0, NE;
            long long eb;
            bool hl;
            const int R = tile_rows(T, q, S, &r0, &eb, &NE, &hl);
            if (R == 0) continue;
            for (int i = threadIdx.x; i < NE; i += blockDim.x) S.buf[i] = col[eb + i];
            __syncthreads();
            int u[GC_PER], rk[GC_PER];
            const int nv = thread_entries(S, R, NE, u, rk);
            unsigned m = 0;
#pragma unroll
            for (int k = 0; k < GC_PER; ++k) m |= (k < nv && u[k] >= lo && u[k] < hi ? 1u : 0u) << k;
            ull total;
            const ull prefix = block_excl_scan((ull)__popc(m), S.w, &total);
            record_bases(S, R, NE, nv, prefix, total, m, 0u, 0u);
            __syncthreads();
            for (int r = threadIdx.x; r < R; r += blockDim.x) {
                if (hl && r == R - 1) continue;  // the heavy row: its segments
                cnt[r0 + r] = (long long)(f16(S.base[r + 1], 0) - f16(S.base[r], 0));
            }
        } else {
            const long long sg = q - nt;
            const int v = T.seg_row[sg], j = T.seg_j[sg];
            const long long rs = T.rp[v], d = T.rp[v + 1] - rs;
            const long long e0 = rs + (long long)j * GC_SEG;
            const int len = (int)std::min<long long>(GC_SEG, d - (long long)j * GC_SEG);
            ull c = 0;
#pragma unroll
            for (int k = 0; k < GC_PER; ++k) {
                const int i = threadIdx.x + k * GC_BLOCK;
                const int x = i < len ? col[e0 + i] : -1;
                c += (x >= lo && x < hi) ? 1ull : 0ull;
            }
            const ull tot = block_sum(c, S.w);
            if (threadIdx.x == 0) {
                segc[sg] = tot;
                if (tot) atomicAdd(reinterpret_cast<ull*>(cnt + v), tot);
            }
        }
        __syncthreads();
    }
}

// pass 2: the entries in range to tcol[trp[v] ...], in row order
__global__ void __launch_bounds__(GC_BLOCK) k_filt_fill(Tiles T, const int* col, int lo, int hi, const long long* trp,
                                                        int* tcol, const ull* segc) {
    __shared__ TileLdsP S;
    __shared__ ull s_pre;
    const long long nt = T.ntiles, ns = nseg_of(T);
    for (long long q = blockIdx.x; q < nt + ns; q += gridDim.x) {
        if (q < nt) {
            int r0, NE;
            long long eb;
            bool hl;
            const int R = tile_rows(T, q, S, &r0, &eb, &NE, &hl);
            if (R == 0) continue;
            for (int i = threadIdx.x; i < NE; i += blockDim.x) S.buf[i] = col[eb + i];
            __syncthreads();
            int u[GC_PER], rk[GC_PER];
            const int nv = thread_entries(S, R, NE, u, rk);
            unsigned m = 0;
#pragma unroll
            for (int k = 0; k < GC_PER; ++k) m |= (k < nv && u[k] >= lo && u[k] < hi ? 1u : 0u) << k;
            ull total;
            const ull prefix = block_excl_scan((ull)__popc(m), S.w, &total);
            record_bases(S, R, NE, nv, prefix, total, m, 0u, 0u);
            __syncthreads();
#pragma unroll
            for (int k = 0; k < GC_PER; ++k) {
                const unsigned bit = 1u << k;
                if (!(m & bit)) continue;
                const int r = rk[k];
                const unsigned rank = (unsigned)prefix + __popc(m & (bit - 1u)) - f16(S.base[r], 0);
                tcol[trp[r0 + r] + rank] = u[k];
            }
        } else {
            const long long sg = q - nt;
            const int v = T.seg_row[sg], j = T.seg_j[sg];
            const long long rs = T.rp[v], d = T.rp[v + 1] - rs;
            const long long e0 = rs + (long long)j * GC_SEG;
            const int len = (int)std::min<long long>(GC_SEG, d - (long long)j * GC_SEG);
            if (threadIdx.x < GC_WAVE) {  // the row's earlier segments' entries in range
                ull a = 0;
                for (long long i = sg - j + threadIdx.x; i < sg; i += GC_WAVE) a += segc[i];
                a = gc_wave_sum(a);
                if (threadIdx.x == 0) s_pre = a;
            }
            for (int i = threadIdx.x; i < len; i += blockDim.x) S.buf[i] = col[e0 + i];
            __syncthreads();
            const int j0 = threadIdx.x * GC_PER;  // this thread's consecutive entries: row order
            unsigned m = 0;
            int u[GC_PER];
#pragma unroll
            for (int k = 0; k < GC_PER; ++k) {
                u[k] = j0 + k < len ? S.buf[j0 + k] : -1;
                m |= (u[k] >= lo && u[k] < hi ? 1u : 0u) << k;
            }
            ull total;
            const ull prefix = block_excl_scan((ull)__popc(m), S.w, &total);
            const long long base = trp[v] + (long long)s_pre + (long long)prefix;
#pragma unroll
            for (int k = 0; k < GC_PER; ++k)
                if (m & (1u << k)) tcol[base + __popc(m & ((1u << k) - 1u))] = u[k];
        }
        __syncthreads();
    }
}

int small_grid(long long items) {
    return (int)std::max<long long>(1, std::min<long long>((items + GC_BLOCK - 1) / GC_BLOCK, 8192));
}

Tiles tiles_of(const gc_graph* g) {
    Tiles T;
    T.rp = g->rp;
    T.r0 = g->tile_r0;
    T.ntiles = g->ntiles;
    T.seg_base = g->seg_base;
    T.seg_row = g->seg_row;
    T.seg_j = g->seg_j;
    T.n = (int)g->n;
    return T;
}

int prep_grid(const gc_graph* g) {
    return (int)std::max<long long>(1, std::min<long long>(g->ntiles + g->nseg_cap, GC_PREP_GRID));
}

}  // namespace

// The tiling is built into locals and published to g only once every allocation and
// kernel succeeded: a failure leaves g without a tiling (the next call retries) instead of
// a half-built one that later passes would launch with.
int gc_build_tiling(gc_graph* g) {
    if (g->tile_r0) return GC_OK;
    const hipStream_t s = g->stream;
    const long long n = g->n, nnz = g->nnz;
    const long long ntiles = (nnz + n + GC_TW - 1) / GC_TW;
    const long long nseg_cap = nnz / GC_SEG + nnz / GC_TH + 1;
    int* tile_r0 = nullptr;
    long long* seg_base = nullptr;
    int *seg_row = nullptr, *seg_j = nullptr;
    ull* seg_aux = nullptr;
    unsigned* seg_cls = nullptr;
    long long* cnt = nullptr;
    auto release = [&]() {
        for (void* p : {(void*)tile_r0, (void*)seg_base, (void*)seg_row, (void*)seg_j, (void*)seg_aux, (void*)seg_cls})
            if (p) gc_dfree(p);
    };
    int rc = GC_OK;
    if (gc_dmalloc((void**)&tile_r0, sizeof(int) * (size_t)(ntiles + 1)) != hipSuccess ||
        gc_dmalloc((void**)&seg_base, sizeof(long long) * (size_t)(ntiles + 1)) != hipSuccess ||
        gc_dmalloc((void**)&seg_row, sizeof(int) * (size_t)nseg_cap) != hipSuccess ||
        gc_dmalloc((void**)&seg_j, sizeof(int) * (size_t)nseg_cap) != hipSuccess ||
        gc_dmalloc((void**)&seg_aux, sizeof(ull) * (size_t)nseg_cap) != hipSuccess ||
        gc_dmalloc((void**)&seg_cls, sizeof(unsigned) * (size_t)nseg_cap * GC_BLOCK) != hipSuccess ||
        gc_dmalloc((void**)&cnt, sizeof(long long) * (size_t)(ntiles + 1)) != hipSuccess) {
        if (cnt) gc_dfree(cnt);
        release();
        gc_set_error("gc_build_tiling: device allocation failed");
        return GC_ENOMEM;
    }
    hipLaunchKernelGGL(k_tile_bounds, dim3(small_grid(ntiles + 1)), dim3(GC_BLOCK), 0, s, g->rp, n, ntiles, tile_r0);
    hipLaunchKernelGGL(k_tile_nseg, dim3(small_grid(ntiles + 1)), dim3(GC_BLOCK), 0, s, g->rp, (const int*)tile_r0,
                       ntiles, cnt);
    rc = scan_ll(cnt, seg_base, ntiles + 1, s);
    if (rc == GC_OK)
        hipLaunchKernelGGL(k_tile_segs, dim3(small_grid(ntiles)), dim3(GC_BLOCK), 0, s, (const int*)tile_r0, ntiles,
                           (const long long*)seg_base, seg_row, seg_j);
    const hipError_t se = hipStreamSynchronize(s);
    const hipError_t le = hipGetLastError();
    gc_dfree(cnt);
    if (rc == GC_OK && (se != hipSuccess || le != hipSuccess)) {
        gc_set_error("gc_build_tiling: %s", hipGetErrorString(se != hipSuccess ? se : le));
        rc = GC_EHIP;
    }
    if (rc) {
        release();
        return rc;
    }
    g->ntiles = ntiles;
    g->nseg_cap = nseg_cap;
    g->tile_r0 = tile_r0;
    g->seg_base = seg_base;
    g->seg_row = seg_row;
    g->seg_j = seg_j;
    g->seg_aux = seg_aux;
    g->seg_cls = seg_cls;
    return GC_OK;
}

bool gc_partition_hubflags_supported() { return GC_PART_HUBFLAG; }

// v's in-rows (v->trp, v->tcol) for the vertex range [lo, hi) of the symmetric graph g whose
// rows v borrows (k_filt_count / k_filt_fill over g's tiling), on v's stream
int gc_filter_rows_sym(gc_graph* g, gc_graph* v, long long lo, long long hi) {
    const hipStream_t s = v->stream;
    const long long n = g->n;
    GC_HIP(gc_dmalloc((void**)&v->trp, sizeof(long long) * (size_t)(n + 1)));
    if (n == 0 || g->nnz == 0) {
        GC_HIP(hipMemsetAsync(v->trp, 0, sizeof(long long) * (size_t)(n + 1), s));
        GC_HIP(gc_dmalloc((void**)&v->tcol, sizeof(int)));
        GC_HIP(hipStreamSynchronize(s));
        return GC_OK;
    }
    int rc = gc_build_tiling(g);
    if (rc) return rc;
    const Tiles T = tiles_of(g);
    long long* cnt = nullptr;
    ull* segc = nullptr;
    GC_HIP(gc_dmalloc((void**)&cnt, sizeof(long long) * (size_t)(n + 1)));
    if (gc_dmalloc((void**)&segc, sizeof(ull) * (size_t)std::max<long long>(g->nseg_cap, 1)) != hipSuccess) {
        gc_dfree(cnt);
        gc_set_error("gc_filter_rows_sym: device allocation failed");
        return GC_ENOMEM;
    }
    GC_HIP(hipMemsetAsync(cnt, 0, sizeof(long long) * (size_t)(n + 1), s));
    const int grid = prep_grid(g);
    hipLaunchKernelGGL(k_filt_count, dim3(grid), dim3(GC_BLOCK), 0, s, T, (const int*)g->col, (int)lo, (int)hi, cnt,
                       segc);
    rc = scan_ll(cnt, v->trp, n + 1, s);
    gc_dfree(cnt);
    long long e = 0;
    if (!rc) rc = gc_read_dev(s, &e, (const long long*)v->trp + n, 1);
    if (!rc && gc_dmalloc((void**)&v->tcol, sizeof(int) * (size_t)std::max<long long>(e, 1)) != hipSuccess) {
        gc_set_error("gc_filter_rows_sym: allocation of %lld in-entries failed", e);
        rc = GC_ENOMEM;
    }
    if (!rc) {
        hipLaunchKernelGGL(k_filt_fill, dim3(grid), dim3(GC_BLOCK), 0, s, T, (const int*)g->col, (int)lo, (int)hi,
                           (const long long*)v->trp, v->tcol, (const ull*)segc);
        const hipError_t le = hipGetLastError(), se = hipStreamSynchronize(s);
        if (le != hipSuccess || se != hipSuccess) {
            gc_set_error("gc_filter_rows_sym: %s", hipGetErrorString(le != hipSuccess ? le : se));
            rc = GC_EHIP;
        }
    }
    hipStreamSynchronize(s);
    gc_dfree(segc);
    return rc;
}

int gc_partition(gc_graph* g, const int* src, int* dst, int prio, uint64_t seed, ull* bad, unsigned char* hubflag,
                 int hub_t) {
    if (g->n == 0 || g->nnz == 0) {
        if (g->n) {
            GC_HIP(hipMemsetAsync(g->nlow, 0, sizeof(int) * (size_t)g->n, g->stream));
            if (g->neq) GC_HIP(hipMemsetAsync(g->neq, 0, sizeof(int) * (size_t)g->n, g->stream));
            if (g->nhe) GC_HIP(hipMemsetAsync(g->nhe, 0, sizeof(int) * (size_t)g->n, g->stream));
        }
        return GC_OK;
    }
    int rc = gc_build_tiling(g);
    if (rc) return rc;
    PartArgs a;
    a.T = tiles_of(g);
    a.src = src;
    a.dst = dst;
    a.deg = g->deg;
    a.kb = g->kb;
    a.nlow = g->nlow;
    a.neq = g->neq;
    a.nhe = g->nhe;
    a.seed = (ull)seed;
    a.bad = bad;
    a.seg_aux = g->seg_aux;
    a.seg_cls = g->seg_cls;
    a.hflag = (GC_PART_HUBFLAG && !prio && hub_t >= 0) ? hubflag : nullptr;
    a.hub_t = hub_t;
    a.hub_code = hub_t >= 0 ? gc_deg_code((long long)hub_t + 1) : 0u;
    a.hub_amb = hub_t >= 0 && gc_deg_code((long long)hub_t) == a.hub_code;
    const int grid = prep_grid(g);
    if (prio) hipLaunchKernelGGL(k_part1<1>, dim3(grid), dim3(GC_BLOCK), 0, g->stream, a);
    else hipLaunchKernelGGL(k_part1<0>, dim3(grid), dim3(GC_BLOCK), 0, g->stream, a);
    hipLaunchKernelGGL(k_part2, dim3(grid), dim3(GC_BLOCK), 0, g->stream, a);
    GC_HIP(hipGetLastError());
    return GC_OK;
}

int gc_validate_tiles(gc_graph* g, const int* colors, const unsigned char* c8, long long lo, long long hi) {
    if (g->n == 0 || lo >= hi) return GC_OK;
    int rc = gc_build_tiling(g);
    if (rc) return rc;
    // the tiles holding rows [lo, hi): tile t holds the rows with rp[r] + r in [t GC_TW, (t+1) GC_TW)
    VRange V;
    V.lo = (int)lo;
    V.hi = (int)hi;
    if (lo == 0 && hi == g->n) {
        V.t0 = 0;
        V.t1 = g->ntiles;
    } else {
        long long rl = 0, rh = 0;
        GC_HIP(hipMemcpyAsync(&rl, g->rp + lo, sizeof(long long), hipMemcpyDeviceToHost, g->stream));
        GC_HIP(hipMemcpyAsync(&rh, g->rp + hi - 1, sizeof(long long), hipMemcpyDeviceToHost, g->stream));
        GC_HIP(hipStreamSynchronize(g->stream));
        V.t0 = std::min<long long>((rl + lo) / GC_TW, g->ntiles);
        V.t1 = std::min<long long>((rh + hi - 1) / GC_TW + 1, g->ntiles);
    }
    long long sb[2] = {0, 0};
    GC_HIP(hipMemcpyAsync(&sb[0], g->seg_base + V.t0, sizeof(long long), hipMemcpyDeviceToHost, g->stream));
    GC_HIP(hipMemcpyAsync(&sb[1], g->seg_base + V.t1, sizeof(long long), hipMemcpyDeviceToHost, g->stream));
    GC_HIP(hipStreamSynchronize(g->stream));
    V.s0 = sb[0];
    V.s1 = sb[1];
    // symmetric graphs: the low parts only (k_validate_tiles' HALF; GC_VALIDATE_HALF=0 reads every entry)
    const bool half = (g->flags & GC_GRAPH_SYMMETRIC) && g->nlow &&
                      !(getenv("GC_VALIDATE_HALF") && atoi(getenv("GC_VALIDATE_HALF")) == 0);
    const Tiles T = tiles_of(g);
    const int grid = prep_grid(g);
    ull* unc = &g->ctl->uncolored;
    ull* conf = &g->ctl->conflicts;
    const int* nl = g->nlow;
    if (c8 && half)
        hipLaunchKernelGGL((k_validate_tiles<1, 1>), dim3(grid), dim3(GC_BLOCK), 0, g->stream, T, V, (const int*)g->col, colors, c8, nl, unc, conf);
    else if (c8)
        hipLaunchKernelGGL((k_validate_tiles<1, 0>), dim3(grid), dim3(GC_BLOCK), 0, g->stream, T, V, (const int*)g->col, colors, c8, nl, unc, conf);
    else if (half)
        hipLaunchKernelGGL((k_validate_tiles<0, 1>), dim3(grid), dim3(GC_BLOCK), 0, g->stream, T, V, (const int*)g->col, colors, c8, nl, unc, conf);
    else
        hipLaunchKernelGGL((k_validate_tiles<0, 0>), dim3(grid), dim3(GC_BLOCK), 0, g->stream, T, V, (const int*)g->col, colors, c8, nl, unc, conf);
    GC_HIP(hipGetLastError());
    return GC_OK;
}

// the count pass (hubmap / hubpre / hperm / hid ready): the entry bits and their word
// prefix (kept on g until the fill), hin_rp (n + 1: the exclusive prefix itself) and klow
// (H + 1, zeroed here)
int gc_hub_transpose_sym(gc_graph* g, long long H, long long* hin_rp, long long* klow, int T) {
    const hipStream_t s = g->stream;
    const long long n = g->n, nnz = g->nnz;
    const long long nw = (nnz + 63) / 64;
    gc_hub_bits_free(g);
    const long long words = (n + 31) / 32;
    GC_HIP(gc_dmalloc((void**)&g->hb_mp, sizeof(uint2) * (size_t)std::max<long long>(words, 1)));
    if (words > 0)
        hipLaunchKernelGGL(k_hb_mp, dim3(small_grid(words)), dim3(GC_BLOCK), 0, s, (const unsigned*)g->hubmap,
                           (const unsigned*)g->hubpre, words, g->hb_mp);
    GC_HIP(gc_dmalloc((void**)&g->hb_bits, sizeof(ull) * (size_t)(nw + 1)));
    GC_HIP(gc_dmalloc((void**)&g->hb_wpre, sizeof(long long) * (size_t)(nw + 1)));
    long long* wcnt = nullptr;
    GC_HIP(gc_dmalloc((void**)&wcnt, sizeof(long long) * (size_t)(nw + 1)));
    GC_HIP(hipMemsetAsync(g->hb_bits + nw, 0, sizeof(ull), s));  // rank(nnz) may read word nw
    GC_HIP(hipMemsetAsync(wcnt + nw, 0, sizeof(long long), s));
    GC_HIP(hipMemsetAsync(klow, 0, sizeof(long long) * (size_t)(H + 1), s));
    const int grid = (int)std::max<long long>(1, std::min<long long>((nw + 255) / 256, 8192));
    // the rank partition marked the hub entries for this threshold (gc_alloc_graph_common):
    // stream its flag bytes; else gather each entry's hub bit
    const bool flags = g->hubflag && g->hubflag_t == T;
    if (nw > 0 && flags)
        hipLaunchKernelGGL(k_hbit_flags, dim3(grid), dim3(GC_BLOCK), 0, s, (const unsigned char*)g->hubflag, nnz,
                           g->hb_bits, wcnt, nw);
    else if (nw > 0)
        hipLaunchKernelGGL(k_hbit, dim3(grid), dim3(GC_BLOCK), 0, s, (const int*)g->col, nnz, n,
                           (const uint2*)g->hb_mp, g->hb_bits, wcnt, nw);
    int rc = scan_ll(wcnt, g->hb_wpre, nw + 1, s);  // (synchronises the stream)
    gc_dfree(wcnt);
    if (g->hubflag) {  // used once: the hub index is kept with the graph
        gc_dfree(g->hubflag);
        g->hubflag = nullptr;
        g->hubflag_t = -1;
    }
    if (rc) return rc;
    hipLaunchKernelGGL(k_hin_rank, dim3(small_grid(n + 1)), dim3(GC_BLOCK), 0, s, (const long long*)g->rp, n,
                       (const ull*)g->hb_bits, (const long long*)g->hb_wpre, (const int*)g->nlow, (const int*)g->hid,
                       hin_rp, klow);
    GC_HIP(hipGetLastError());
    // the caller reads hin_rp[n] with a plain hipMemcpy, which does not wait for this
    // (non-blocking) stream: hin_rp must be final before returning (round 4's first GPU run
    // of this pass read it early, sized hin_col from a stale E and the fill faulted)
    GC_HIP(hipStreamSynchronize(s));
    return GC_OK;
}

// fill pass (hin_rp / hin_col allocated), then hlow rows as klow-prefixes (hlow_rp ready);
// the entry bits are released
int gc_hub_transpose_fill(gc_graph* g, long long H) {
    const hipStream_t s = g->stream;
    const long long nw = (g->nnz + 63) / 64;
    if (!g->hb_bits || !g->hb_wpre || !g->hb_mp) { gc_set_error("gc_hub_transpose_fill: no entry bits"); return GC_EINVAL; }
    const int grid = (int)std::max<long long>(1, std::min<long long>((nw + 255) / 256, 8192));
    if (nw > 0)
        hipLaunchKernelGGL(k_hin_fill, dim3(grid), dim3(GC_BLOCK), 0, s, (const int*)g->col, nw, (const ull*)g->hb_bits,
                           (const long long*)g->hb_wpre, (const uint2*)g->hb_mp, (const int*)g->hperm, g->hin_col);
    if (H > 0)
        hipLaunchKernelGGL(k_hlow_copy, dim3((int)std::min<long long>((H + 3) / 4, 8192)), dim3(GC_BLOCK), 0, s,
                           (const int*)g->hub_v, H, (const long long*)g->hin_rp, (const int*)g->hin_col,
                           (const long long*)g->hlow_rp, g->hlow_col);
    GC_HIP(hipGetLastError());
    GC_HIP(hipStreamSynchronize(s));  // the bits go back to the cache idle
    gc_hub_bits_free(g);
    return GC_OK;
}

void gc_hub_bits_free(gc_graph* g) {
    if (g->hb_bits) gc_dfree(g->hb_bits);
    if (g->hb_wpre) gc_dfree(g->hb_wpre);
    if (g->hb_mp) gc_dfree(g->hb_mp);
    g->hb_bits = nullptr;
    g->hb_wpre = nullptr;
    g->hb_mp = nullptr;
}
