/*
 * gcolor_omp.c -- multi-threaded CPU restatement of variant A (coloring.py:73-132).
 *
 * BENCHMARK BASELINE ONLY (SURVEY.md §8d "C++/OpenMP restatement on all
 * host cores").  Only bench.py's cpu_baseline leg and tests/ load this library; the
 * product path never links or calls it.  tests/test_oracle_omp.py checks it bit-exact
 * (colours and every per-round record) against gcolor_oracle.c on the golden set and on
 * seeded R-MAT / uniform graphs.
 *
 * Same semantics as gcolor_oracle.c (which cites the reference line by line):
 *   init / seed   coloring.py:12-35    deg 0 -> colour 0; argmax (deg, pos) -> colour 0
 *   round         coloring.py:80-130   frontier = uncoloured with a coloured LISTED
 *                                      neighbour; mex of their colours (coloring.py:44-54);
 *                                      per-colour LFMIS under rank (deg, pos) (coloring.py:
 *                                      56-70); winners take their candidate
 *   E1            SURVEY.md §8a a7     zero proposers, uncoloured left: one argmax seed per
 *                                      component of the uncoloured-induced subgraph
 * but organised for many cores instead of as the reference's per-round full scans:
 *   - the frontier is pushed: a vertex coloured this round claims the vertices that list
 *     it (their in-row), so a round touches only the frontier's rows;
 *   - the LFMIS is computed by Jones-Plassmann sweeps (a vertex is IN once every
 *     same-candidate lower-rank listed neighbour is OUT, OUT once one is IN), whose
 *     fixpoint is the lexicographically-first MIS -- independent of thread timing;
 *   - hubs (deg > HUB_T) keep a forbidden-colour bitmap pushed by their neighbours'
 *     commits instead of re-reading their rows each round, and sit out the light
 *     vertices' sweeps (every hub ranks above every light vertex, so no light vertex waits
 *     on a hub): a light winner flags the hubs listing it that propose its colour, then
 *     the remaining hubs run JP among themselves over their lower-rank hub entries.
 * Every thread-shared byte is read and written with relaxed atomics.
 */
#include <omp.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OMP_OK 0
#define OMP_ENOMEM (-1)
#define OMP_EROUNDS (-2)

#define HUB_T 512
#define HUB_W 128 /* bitmap words per hub: colours < 4096 */

#define ST_UND 0
#define ST_IN 1
#define ST_OUT 2

static inline int rank_lt(const int32_t* deg, int64_t u, int64_t v) {
    return deg[u] < deg[v] || (deg[u] == deg[v] && u < v);
}
static inline uint8_t ld8(const uint8_t* p) { return __atomic_load_n(p, __ATOMIC_RELAXED); }
static inline void st8(uint8_t* p, uint8_t v) { __atomic_store_n(p, v, __ATOMIC_RELAXED); }
static inline int32_t ld32(const int32_t* p) { return __atomic_load_n(p, __ATOMIC_RELAXED); }
static inline void st32(int32_t* p, int32_t v) { __atomic_store_n(p, v, __ATOMIC_RELAXED); }

typedef struct {
    int64_t n;
    const int64_t* rp;
    const int32_t* col;
    const int64_t* trp; /* in-rows (== rp/col when symmetric) */
    const int32_t* tcol;
    int32_t* deg;
    int32_t* color;
    int32_t* cround;
    int32_t* cand;
    int32_t* pround;  /* round in which v last proposed */
    uint8_t* st;      /* JP state of this round */
    uint8_t* inF;     /* claimed: coloured or in the frontier */
    int32_t* hid;     /* hub index or -1 */
    int64_t nh;
    int32_t* hub_v;
    uint32_t* hbits;
    uint8_t* hkill;
    int64_t* hlow_rp; /* lower-rank hubs of each hub row (hub indices) */
    int32_t* hlow;
} G;

/* per-thread append buffers merged into one list */
typedef struct {
    int32_t* a;
    int64_t n, cap;
} Buf;
static int buf_push(Buf* b, int32_t v) {
    if (b->n == b->cap) {
        int64_t c = b->cap ? 2 * b->cap : 1024;
        int32_t* p = (int32_t*)realloc(b->a, sizeof(int32_t) * (size_t)c);
        if (!p) return -1;
        b->a = p;
        b->cap = c;
    }
    b->a[b->n++] = v;
    return 0;
}
/* concatenate the nt thread buffers into out (out must hold the total); returns count */
static int64_t merge(Buf* bufs, int nt, int32_t* out) {
    int64_t o = 0;
    for (int t = 0; t < nt; ++t) {
        if (bufs[t].n) memcpy(out + o, bufs[t].a, sizeof(int32_t) * (size_t)bufs[t].n);  /* (a may be NULL) */
        o += bufs[t].n;
        bufs[t].n = 0;
    }
    return o;
}

/* colour u with c and push: hubs listing u get bit c, uncoloured vertices listing u are
   claimed into the next frontier (thread buffer b) */
static int colour_push(G* g, int32_t u, int32_t c, int32_t round, Buf* b) {
    st32(&g->color[u], c);
    if (g->cround) g->cround[u] = round;
    for (int64_t e = g->trp[u]; e < g->trp[u + 1]; ++e) {
        const int32_t x = g->tcol[e];
        const int32_t hx = g->hid[x];
        if (hx >= 0 && c < 32 * HUB_W) {
            uint32_t* w = &g->hbits[(int64_t)hx * HUB_W + (c >> 5)];
            const uint32_t bit = 1u << (c & 31);
            if (!(__atomic_load_n(w, __ATOMIC_RELAXED) & bit)) __atomic_fetch_or(w, bit, __ATOMIC_RELAXED);
        }
        if (ld8(&g->inF[x])) continue;
        if (__atomic_exchange_n(&g->inF[x], (uint8_t)1, __ATOMIC_RELAXED) == 0)
            if (buf_push(b, x)) return -1;
    }
    return 0;
}

/* mex of v's coloured listed neighbours; stamp/cap: thread scratch (deg + 2 entries) */
static int64_t mex_scan(const G* g, int32_t v, int64_t* stamp, int64_t sc) {
    for (int64_t e = g->rp[v]; e < g->rp[v + 1]; ++e) {
        const int32_t c = ld32(&g->color[g->col[e]]);
        if (c >= 0 && c <= g->deg[v]) stamp[c] = sc;
    }
    int64_t m = 0;
    while (stamp[m] == sc) ++m;
    return m;
}

/* JP flag of entry u for proposer v with candidate cv: 1 = same-colour IN, 2 = same-colour
   undecided, 0 = irrelevant (not a proposer this round, other colour, or OUT) */
static inline int jp_flag(const G* g, int32_t u, int32_t cv, int32_t round) {
    if (g->pround[u] != round || g->cand[u] != cv) return 0;
    const uint8_t s = ld8(&g->st[u]);
    return s == ST_IN ? 1 : (s == ST_UND ? 2 : 0);
}

int omp_color(const int64_t* rp, const int32_t* col, int64_t n, int32_t symmetric, int32_t nthreads,
              int32_t* color, int32_t* colored_round, int64_t* r_U, int64_t* r_F, int64_t* r_maxmex,
              int64_t* r_acc, int64_t* r_seeds, int64_t cap, int64_t* rounds_out, int64_t* reseeds_out) {
    if (nthreads > 0) omp_set_num_threads(nthreads);
    const int nt = omp_get_max_threads();
    const int64_t nnz = rp[n];
    int status = OMP_OK;
    G g;
    memset(&g, 0, sizeof(g));
    g.n = n;
    g.rp = rp;
    g.col = col;
    g.color = color;
    g.cround = colored_round;
    int64_t* trp_own = NULL;
    int32_t* tcol_own = NULL;
    int32_t *F = NULL, *Fn = NULL, *L0 = NULL, *L1 = NULL, *H0 = NULL, *H1 = NULL, *ulist = NULL;
    int64_t *parent = NULL, *best = NULL;
    Buf* bufs = (Buf*)calloc((size_t)nt, sizeof(Buf));
    int64_t** stamps = (int64_t**)calloc((size_t)nt, sizeof(int64_t*));
    int64_t* scs = (int64_t*)calloc((size_t)nt, sizeof(int64_t));
    const int64_t nn = n > 0 ? n : 1;
    g.deg = (int32_t*)malloc(sizeof(int32_t) * (size_t)nn);
    g.cand = (int32_t*)malloc(sizeof(int32_t) * (size_t)nn);
    g.pround = (int32_t*)malloc(sizeof(int32_t) * (size_t)nn);
    g.st = (uint8_t*)malloc((size_t)nn);
    g.inF = (uint8_t*)malloc((size_t)nn);
    g.hid = (int32_t*)malloc(sizeof(int32_t) * (size_t)nn);
    F = (int32_t*)malloc(sizeof(int32_t) * (size_t)nn);
    Fn = (int32_t*)malloc(sizeof(int32_t) * (size_t)nn);
    L0 = (int32_t*)malloc(sizeof(int32_t) * (size_t)nn);
    L1 = (int32_t*)malloc(sizeof(int32_t) * (size_t)nn);
    H0 = (int32_t*)malloc(sizeof(int32_t) * (size_t)nn);
    H1 = (int32_t*)malloc(sizeof(int32_t) * (size_t)nn);
    if (!bufs || !stamps || !scs || !g.deg || !g.cand || !g.pround || !g.st || !g.inF || !g.hid || !F || !Fn || !L0 ||
        !L1 || !H0 || !H1) {
        status = OMP_ENOMEM;
        goto out;
    }
    int64_t maxdeg = 0;
#pragma omp parallel for reduction(max : maxdeg) schedule(static)
    for (int64_t v = 0; v < n; ++v) {
        g.deg[v] = (int32_t)(rp[v + 1] - rp[v]);
        if (g.deg[v] > maxdeg) maxdeg = g.deg[v];
        g.pround[v] = -1;
        g.cand[v] = -1;
        g.st[v] = ST_UND;
    }
    for (int t = 0; t < nt; ++t) {
        stamps[t] = (int64_t*)calloc((size_t)maxdeg + 2, sizeof(int64_t));
        if (!stamps[t]) { status = OMP_ENOMEM; goto out; }
    }
    if (symmetric) {
        g.trp = rp;
        g.tcol = col;
    } else {  /* in-rows: who lists u */
        trp_own = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
        tcol_own = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nnz > 0 ? nnz : 1));
        if (!trp_own || !tcol_own) { status = OMP_ENOMEM; goto out; }
        for (int64_t e = 0; e < nnz; ++e) trp_own[col[e] + 1]++;
        for (int64_t v = 0; v < n; ++v) trp_own[v + 1] += trp_own[v];
        for (int64_t v = 0; v < n; ++v)
            for (int64_t e = rp[v]; e < rp[v + 1]; ++e) tcol_own[trp_own[col[e]]++] = (int32_t)v;
        for (int64_t v = n; v > 0; --v) trp_own[v] = trp_own[v - 1];
        trp_own[0] = 0;
        g.trp = trp_own;
        g.tcol = tcol_own;
    }
    /* hubs */
    g.nh = 0;
    for (int64_t v = 0; v < n; ++v) g.hid[v] = g.deg[v] > HUB_T ? (int32_t)g.nh++ : -1;
    if (g.nh) {
        g.hub_v = (int32_t*)malloc(sizeof(int32_t) * (size_t)g.nh);
        g.hbits = (uint32_t*)calloc((size_t)g.nh * HUB_W, sizeof(uint32_t));
        g.hkill = (uint8_t*)calloc((size_t)g.nh, 1);
        g.hlow_rp = (int64_t*)calloc((size_t)g.nh + 1, sizeof(int64_t));
        if (!g.hub_v || !g.hbits || !g.hkill || !g.hlow_rp) { status = OMP_ENOMEM; goto out; }
        for (int64_t v = 0; v < n; ++v)
            if (g.hid[v] >= 0) g.hub_v[g.hid[v]] = (int32_t)v;
#pragma omp parallel for schedule(dynamic, 16)
        for (int64_t x = 0; x < g.nh; ++x) {
            const int32_t h = g.hub_v[x];
            int64_t k = 0;
            for (int64_t e = rp[h]; e < rp[h + 1]; ++e)
                if (g.hid[col[e]] >= 0 && rank_lt(g.deg, col[e], h)) ++k;
            g.hlow_rp[x + 1] = k;
        }
        for (int64_t x = 0; x < g.nh; ++x) g.hlow_rp[x + 1] += g.hlow_rp[x];
        g.hlow = (int32_t*)malloc(sizeof(int32_t) * (size_t)(g.hlow_rp[g.nh] > 0 ? g.hlow_rp[g.nh] : 1));
        if (!g.hlow) { status = OMP_ENOMEM; goto out; }
#pragma omp parallel for schedule(dynamic, 16)
        for (int64_t x = 0; x < g.nh; ++x) {
            const int32_t h = g.hub_v[x];
            int64_t o = g.hlow_rp[x];
            for (int64_t e = rp[h]; e < rp[h + 1]; ++e)
                if (g.hid[col[e]] >= 0 && rank_lt(g.deg, col[e], h)) g.hlow[o++] = g.hid[col[e]];
        }
    }

    /* init (coloring.py:12-17) + seed (coloring.py:19-35) */
    int64_t U = 0;
#pragma omp parallel for reduction(+ : U) schedule(static)
    for (int64_t v = 0; v < n; ++v) {
        color[v] = g.deg[v] == 0 ? 0 : -1;
        if (colored_round) colored_round[v] = color[v];
        g.inF[v] = color[v] == 0;
        U += color[v] == -1;
    }
    int64_t s = -1;
    for (int64_t v = 0; v < n; ++v)
        if (color[v] == -1 && (s < 0 || g.deg[v] >= g.deg[s])) s = v;
    if (s >= 0) {
        color[s] = 0;
        if (colored_round) colored_round[s] = 0;
        g.inF[s] = 1;
        U--;
    }
    /* first frontier and hub bitmaps: one pass (covers isolated vertices listed by others) */
    int64_t nF = 0;
    {
#pragma omp parallel
        {
            Buf* b = &bufs[omp_get_thread_num()];
#pragma omp for schedule(dynamic, 1024)
            for (int64_t v = 0; v < n; ++v) {
                const int32_t hx = g.hid[v];
                if (hx >= 0)  /* hub bitmap: colours of its coloured listed neighbours */
                    for (int64_t e = rp[v]; e < rp[v + 1]; ++e) {
                        const int32_t c = color[col[e]];
                        if (c >= 0 && c < 32 * HUB_W) g.hbits[(int64_t)hx * HUB_W + (c >> 5)] |= 1u << (c & 31);
                    }
                if (color[v] != -1) continue;
                int any = 0;
                for (int64_t e = rp[v]; e < rp[v + 1] && !any; ++e) any = color[col[e]] >= 0;
                if (any) {
                    g.inF[v] = 1;
                    buf_push(b, (int32_t)v);
                }
            }
        }
        nF = merge(bufs, nt, F);
    }

    int64_t reseeds = 0;
    int64_t r = 0;
    for (;; ++r) {
        if (r >= cap && (r_U || r_F || r_maxmex || r_acc || r_seeds)) { status = OMP_EROUNDS; break; }
        if (r_U) r_U[r] = U;
        if (r_F) r_F[r] = nF;
        if (r_maxmex) r_maxmex[r] = -1;
        if (r_acc) r_acc[r] = 0;
        if (r_seeds) r_seeds[r] = 0;
        if (U == 0) { ++r; break; }
        if (nF == 0) { /* E1 (sequential union-find, as gcolor_oracle.c) */
            if (!ulist) {
                ulist = (int32_t*)malloc(sizeof(int32_t) * (size_t)nn);
                parent = (int64_t*)malloc(sizeof(int64_t) * (size_t)nn);
                best = (int64_t*)malloc(sizeof(int64_t) * (size_t)nn);
                if (!ulist || !parent || !best) { status = OMP_ENOMEM; break; }
            }
            int64_t nu = 0;
            for (int64_t v = 0; v < n; ++v)
                if (color[v] == -1) { ulist[nu++] = (int32_t)v; parent[v] = v; best[v] = -1; }
            for (int64_t i = 0; i < nu; ++i) {
                const int64_t v = ulist[i];
                for (int64_t e = rp[v]; e < rp[v + 1]; ++e) {
                    const int64_t u = col[e];
                    if (color[u] != -1) continue;
                    int64_t a = v, b2 = u;
                    while (parent[a] != a) { parent[a] = parent[parent[a]]; a = parent[a]; }
                    while (parent[b2] != b2) { parent[b2] = parent[parent[b2]]; b2 = parent[b2]; }
                    if (a != b2) { if (a < b2) parent[b2] = a; else parent[a] = b2; }
                }
            }
            for (int64_t i = 0; i < nu; ++i) {
                const int64_t v = ulist[i];
                int64_t a = v;
                while (parent[a] != a) a = parent[a];
                if (best[a] < 0 || g.deg[v] >= g.deg[best[a]]) best[a] = v;
            }
            int64_t ns = 0;
            Buf* b = &bufs[0];
            for (int64_t i = 0; i < nu; ++i) {
                const int64_t v = ulist[i];
                if (parent[v] == v && best[v] >= 0) {
                    const int32_t sd = (int32_t)best[v];
                    g.inF[sd] = 1;
                    if (colour_push(&g, sd, 0, (int32_t)(r + 1), b)) { status = OMP_ENOMEM; break; }
                    ++ns;
                }
            }
            if (status) break;
            /* the claimed list may hold a seed coloured after it was claimed: drop coloured */
            int64_t m = 0;
            for (int64_t i = 0; i < b->n; ++i)
                if (color[b->a[i]] == -1) F[m++] = b->a[i];
            b->n = 0;
            nF = m;
            reseeds += ns;
            if (r_seeds) r_seeds[r] = ns;
            U -= ns;
            continue;
        }

        /* propose (coloring.py:44-54): colours as at the round start -- winners are
           written only after the resolution */
        int64_t maxmex = -1, nl = 0, nhp = 0;
        {
            const int32_t rr = (int32_t)r;
#pragma omp parallel reduction(max : maxmex)
            {
                const int t = omp_get_thread_num();
                int64_t* stamp = stamps[t];
#pragma omp for schedule(dynamic, 256)
                for (int64_t i = 0; i < nF; ++i) {
                    const int32_t v = F[i];
                    const int32_t hx = g.hid[v];
                    int64_t m = -1;
                    if (hx >= 0) {
                        const uint32_t* hb = &g.hbits[(int64_t)hx * HUB_W];
                        for (int w = 0; w < HUB_W; ++w)
                            if (~hb[w]) { m = 32ll * w + __builtin_ctz(~hb[w]); break; }
                        g.hkill[hx] = 0;
                    }
                    if (m < 0) m = mex_scan(&g, v, stamp, ++scs[t]);
                    g.cand[v] = (int32_t)m;
                    g.pround[v] = rr;
                    g.st[v] = ST_UND;
                    if (m > maxmex) maxmex = m;
                }
            }
        }
        if (r_maxmex) r_maxmex[r] = maxmex;
        /* split: lights (sweep list) / hubs */
        for (int64_t i = 0; i < nF; ++i) {
            if (g.hid[F[i]] >= 0) H0[nhp++] = F[i];
            else L0[nl++] = F[i];
        }
        /* JP over the lights; lower-rank light entries only (a light's lower-rank entries
           are light) */
        const int32_t rr = (int32_t)r;
        int32_t *Li = L0, *Lo = L1;
        /* GC_OMP_SWEEPLOG: per round, the JP list sizes (lights, then hubs) on stderr --
           the shape of the dependency chains the GPU's sweeps walk (analysis only) */
        static int slog = -1;
        if (slog < 0) slog = getenv("GC_OMP_SWEEPLOG") != NULL;
        if (slog) fprintf(stderr, "r %lld F %lld L", (long long)r, (long long)nF);
        while (nl > 0) {
            if (slog) fprintf(stderr, " %lld", (long long)nl);
#pragma omp parallel
            {
                Buf* b = &bufs[omp_get_thread_num()];
#pragma omp for schedule(dynamic, 256)
                for (int64_t i = 0; i < nl; ++i) {
                    const int32_t v = Li[i];
                    const int32_t cv = g.cand[v];
                    int f = 0;
                    for (int64_t e = rp[v]; e < rp[v + 1]; ++e) {
                        const int32_t u = col[e];
                        if (!rank_lt(g.deg, u, v)) continue;
                        f |= jp_flag(&g, u, cv, rr);
                        if (f & 1) break;
                    }
                    if (f & 1) st8(&g.st[v], ST_OUT);
                    else if (f & 2) buf_push(b, v);
                    else st8(&g.st[v], ST_IN);
                }
            }
            nl = merge(bufs, nt, Lo);
            int32_t* t = Li;
            Li = Lo;
            Lo = t;
        }
        /* hubs: flags from the light winners, then JP among the hubs (hlow entries) */
        if (nhp) {
/* a light winner flags every hub listing it (its in-row) that proposes its colour */
#pragma omp parallel for schedule(dynamic, 256)
            for (int64_t i = 0; i < nF; ++i) {
                const int32_t w = F[i];
                if (g.hid[w] >= 0 || ld8(&g.st[w]) != ST_IN) continue;
                const int32_t cw = g.cand[w];
                for (int64_t e = g.trp[w]; e < g.trp[w + 1]; ++e) {
                    const int32_t x = g.tcol[e];
                    const int32_t hx = g.hid[x];
                    if (hx >= 0 && g.pround[x] == rr && g.cand[x] == cw) st8(&g.hkill[hx], 1);
                }
            }
            int32_t *Hi = H0, *Ho = H1;
            int64_t nh = nhp;
            if (slog) fprintf(stderr, " H");
            while (nh > 0) {
                if (slog) fprintf(stderr, " %lld", (long long)nh);
#pragma omp parallel
                {
                    Buf* b = &bufs[omp_get_thread_num()];
#pragma omp for schedule(dynamic, 16)
                    for (int64_t i = 0; i < nh; ++i) {
                        const int32_t h = Hi[i];
                        const int32_t x = g.hid[h];
                        int f = g.hkill[x] ? 1 : 0;
                        const int32_t ch = g.cand[h];
                        for (int64_t e = g.hlow_rp[x]; e < g.hlow_rp[x + 1] && !(f & 1); ++e)
                            f |= jp_flag(&g, g.hub_v[g.hlow[e]], ch, rr);
                        if (f & 1) st8(&g.st[h], ST_OUT);
                        else if (f & 2) buf_push(b, h);
                        else st8(&g.st[h], ST_IN);
                    }
                }
                nh = merge(bufs, nt, Ho);
                int32_t* t = Hi;
                Hi = Ho;
                Ho = t;
            }
        }
        if (slog) fprintf(stderr, "\n");
        /* commit (coloring.py:114-127) + push; losers stay in the frontier */
        int64_t acc = 0;
#pragma omp parallel reduction(+ : acc)
        {
            Buf* b = &bufs[omp_get_thread_num()];
#pragma omp for schedule(dynamic, 256)
            for (int64_t i = 0; i < nF; ++i) {
                const int32_t v = F[i];
                if (ld8(&g.st[v]) == ST_IN) {
                    if (colour_push(&g, v, g.cand[v], (int32_t)(r + 1), b)) continue;
                    ++acc;
                } else {
                    buf_push(b, v);
                }
            }
        }
        /* a vertex claimed by one winner may itself have won this round: drop coloured */
        {
            int64_t o = 0;
            for (int t = 0; t < nt; ++t) {
                for (int64_t i = 0; i < bufs[t].n; ++i)
                    if (ld32(&color[bufs[t].a[i]]) == -1) Fn[o++] = bufs[t].a[i];
                bufs[t].n = 0;
            }
            int32_t* t = F;
            F = Fn;
            Fn = t;
            nF = o;
        }
        if (r_acc) r_acc[r] = acc;
        U -= acc;
    }
    *rounds_out = r;
    *reseeds_out = reseeds;
out:
    if (bufs)
        for (int t = 0; t < nt; ++t) free(bufs[t].a);
    if (stamps)
        for (int t = 0; t < nt; ++t) free(stamps[t]);
    free(bufs);
    free(stamps);
    free(scs);
    free(g.deg); free(g.cand); free(g.pround); free(g.st); free(g.inF); free(g.hid);
    free(g.hub_v); free(g.hbits); free(g.hkill); free(g.hlow_rp); free(g.hlow);
    free(F); free(Fn); free(L0); free(L1); free(H0); free(H1);
    free(ulist); free(parent); free(best);
    free(trp_own); free(tcol_own);
    return status;
}
