/*
 * gcolor_oracle.c -- CPU restatement of the reference's graph-colouring hot path.
 *
 * TEST INFRASTRUCTURE / CHECKER ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library; the product path
 * (distributed-graph-coloring-with-pyspark_amd/) never links or calls it.
 *
 * Parity pinned: tests/test_oracle_golden.py checks every function here against the
 * golden vectors in tests/golden/cases/, which were produced by running the
 * reference's own coloring.py / coloring_optimized.py (tests/golden/make_golden.py).
 *
 * Semantics restated (all file:line into /root/reference):
 *   init         coloring.py:12-17    colour 0 if deg==0 else -1
 *   seed         coloring.py:19-35    argmax over uncoloured of deg, ties -> LAST in file
 *                                     order (left fold, strict '>'); colour 0
 *   round loop   coloring.py:80-130   U_r printed at :89, stop at 0
 *   propose (A)  coloring.py:44-54    v uncoloured with >=1 coloured listed neighbour
 *                                     proposes mex of their colours; mex >= k -> failure
 *   propose (B)  coloring_optimized.py:150-166  every uncoloured v proposes; no coloured
 *                                     neighbour -> 0
 *   fail check   coloring.py:104-108  any -3 -> return (False, state at round start)
 *   resolve (A)  coloring.py:56-70    per candidate colour: members in file order,
 *                                     stable-sorted by deg asc; accept iff no LISTED
 *                                     neighbour already accepted in the group
 *                                     == LFMIS under rank (deg asc, pos asc)
 *   resolve (B)  coloring_optimized.py:120-126,168-184  arrival-order fold, restated as:
 *                                     arriving v admitted iff no admitted u in N(v) with
 *                                     deg(u) >= deg(v); on admission evicts admitted x of
 *                                     the group with v in N(x) and deg(x) < deg(v)
 *   commit       coloring.py:114-127  colour <- candidate for accepted vertices
 *   validate     coloring.py:149-162  #uncoloured, #(v,u in N(v)) with equal colours
 *
 * Extension E1 (the reference spins forever instead, coloring.py:93-95):
 *   a round with uncoloured vertices but zero proposers re-seeds: every connected
 *   component of the subgraph induced by the uncoloured vertices (edges taken in both
 *   directions) gets its argmax-(deg, pos) vertex coloured 0.  Identical to the
 *   reference on every input where the reference terminates.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_OK 0
#define ORC_FAILED 1
#define ORC_STALLED 2
#define ORC_ENOMEM (-1)
#define ORC_EROUNDS (-2)

typedef struct {
    int64_t rounds;        /* rounds executed (number of U_r entries written)          */
    int64_t fail_round;    /* round in which the bounded attempt failed, else -1        */
    int64_t fail_count;    /* #proposers with mex >= k in that round                   */
    int64_t reseeds;       /* E1 seeds planted (excluding the initial seed)            */
    int64_t max_color;     /* max colour in the final state (-1 if none)               */
    double balg_propose;   /* SURVEY §8d algorithmic bytes, per component              */
    double balg_resolve;
    double balg_push;
    double balg_validate;
} orc_summary;

static inline int64_t deg_of(const int64_t* rp, int64_t v) { return rp[v + 1] - rp[v]; }

/* rank order (deg asc, pos asc): coloring.py:64 stable sort of a file-ordered group.
   With seeded priorities (g_key != NULL) the sort key is key[v] = prio_hash(seed, v)
   instead of deg(v): rank (key asc, pos asc). */
static const int64_t* g_rp;
static const uint32_t* g_key;
static inline uint64_t rank_key(int64_t v) { return g_key ? (uint64_t)g_key[v] : (uint64_t)deg_of(g_rp, v); }
static int cmp_rank(const void* a, const void* b) {
    int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    uint64_t dx = rank_key(x), dy = rank_key(y);
    if (dx != dy) return dx < dy ? -1 : 1;
    return x < y ? -1 : (x > y);
}
static inline int rank_lt(int64_t u, int64_t v) {
    uint64_t ku = rank_key(u), kv = rank_key(v);
    return ku < kv || (ku == kv && u < v);
}

/* Seeded 32-bit priority of vertex v (SURVEY.md §8b priority = 1; BASELINE north_star
   "Jones-Plassmann/Luby priority rounds on seeded hash priorities"): the top half of
   splitmix64(seed + (v + 1) * golden gamma).  The GPU computes the same function
   (csrc/gc_priority.hip, k_prio_hash). */
uint32_t prio_hash(uint64_t seed, int64_t v) {
    uint64_t z = seed + 0x9E3779B97F4A7C15ull * (uint64_t)(v + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (uint32_t)(z >> 32);
}

static int64_t uf_find(int64_t* p, int64_t x) {
    while (p[x] != x) { p[x] = p[p[x]]; x = p[x]; }
    return x;
}

/* argmax of (deg, pos) among uncoloured vertices in [0, n): coloring.py:21-22 */
static int64_t seed_vertex(const int64_t* rp, const int32_t* color, int64_t n) {
    int64_t best = -1, bd = -1;
    for (int64_t v = 0; v < n; ++v) {
        if (color[v] != -1) continue;
        int64_t d = deg_of(rp, v);
        if (d >= bd) { bd = d; best = v; }   /* '>=' : ties go to the later vertex */
    }
    return best;
}

/* E1: one seed per component of the uncoloured-induced subgraph. Returns #seeds. */
static int64_t e1_reseed(const int64_t* rp, const int32_t* col, int64_t n, int32_t* color,
                         int32_t* colored_round, int64_t round_next, int64_t* parent, int64_t* best) {
    for (int64_t v = 0; v < n; ++v) { parent[v] = v; best[v] = -1; }
    for (int64_t v = 0; v < n; ++v) {
        if (color[v] != -1) continue;
        for (int64_t e = rp[v]; e < rp[v + 1]; ++e) {
            int64_t u = col[e];
            if (color[u] != -1) continue;
            int64_t a = uf_find(parent, v), b = uf_find(parent, u);
            if (a != b) { if (a < b) parent[b] = a; else parent[a] = b; }
        }
    }
    for (int64_t v = 0; v < n; ++v) {
        if (color[v] != -1) continue;
        int64_t r = uf_find(parent, v);
        int64_t b = best[r];
        if (b < 0 || deg_of(rp, v) >= deg_of(rp, b)) best[r] = v;  /* v increasing: ties -> later */
    }
    int64_t seeds = 0;
    for (int64_t v = 0; v < n; ++v) {
        /* roots are component minima (union by smaller index), and best >= root */
        if (color[v] == -1 && uf_find(parent, v) == v && best[v] >= 0) {
            int64_t s = best[v];
            best[v] = -1;
            color[s] = 0;
            if (colored_round) colored_round[s] = (int32_t)round_next;
            seeds++;
        }
    }
    return seeds;
}

/*
 * oracle_color: run variant A (variant=0) or B (variant=1) with colour bound k
 * (k < 0: unbounded).  Per-round arrays (capacity cap, may be NULL) receive U_r,
 * |F_r|, max mex, #accepted and #seeds planted in that round.
 * colored_round[v] = first round r at whose START v is coloured (0 for init/seed).
 * On a bounded failure the colours are the state at the start of the failing round
 * (coloring.py:108 returns graph_rdd before the join).
 */
static int color_impl(const int64_t* rp, const int32_t* col, int64_t n, int32_t variant, int64_t k,
                      int32_t e1, const uint32_t* key, int32_t speculative, int32_t* color, int32_t* colored_round,
                      int64_t* r_U, int64_t* r_F, int64_t* r_maxmex, int64_t* r_acc, int64_t* r_seeds,
                      int64_t cap, orc_summary* sum) {
    memset(sum, 0, sizeof(*sum));
    sum->fail_round = -1;
    int status = ORC_OK;
    int64_t* cand = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    int64_t* stamp = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 2));
    int64_t* acc_stamp = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    int64_t* props = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    int64_t* unc = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    int64_t* parent = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    int64_t* best = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    int64_t* trp = NULL;
    int32_t* tcol = NULL;
    if (!cand || !stamp || !acc_stamp || !props || !unc || !parent || !best) { status = ORC_ENOMEM; goto out; }
    if (variant == 1) {   /* in-neighbour lists for variant B's eviction step */
        trp = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
        tcol = (int32_t*)malloc(sizeof(int32_t) * (size_t)(rp[n] > 0 ? rp[n] : 1));
        if (!trp || !tcol) { status = ORC_ENOMEM; goto out; }
        for (int64_t e = 0; e < rp[n]; ++e) trp[col[e] + 1]++;
        for (int64_t v = 0; v < n; ++v) trp[v + 1] += trp[v];
        for (int64_t v = 0; v < n; ++v)
            for (int64_t e = rp[v]; e < rp[v + 1]; ++e) tcol[trp[col[e]]++] = (int32_t)v;
        for (int64_t v = n; v > 0; --v) trp[v] = trp[v - 1];
        trp[0] = 0;
    }
    for (int64_t i = 0; i < n + 2; ++i) stamp[i] = -1;
    for (int64_t v = 0; v < n; ++v) { acc_stamp[v] = -1; cand[v] = -1; }

    /* init (coloring.py:12-17) and seed (coloring.py:19-35) */
    for (int64_t v = 0; v < n; ++v) {
        color[v] = deg_of(rp, v) == 0 ? 0 : -1;
        if (colored_round) colored_round[v] = color[v] == 0 ? 0 : -1;
    }
    int64_t s = seed_vertex(rp, color, n);
    if (s >= 0) {
        color[s] = 0;
        if (colored_round) colored_round[s] = 0;
        sum->balg_push += 16.0 + 8.0 * (double)deg_of(rp, s);
    }
    int64_t nunc = 0;
    for (int64_t v = 0; v < n; ++v) if (color[v] == -1) unc[nunc++] = v;

    int64_t stampc = 0;
    g_rp = rp;
    g_key = key;
    for (int64_t r = 0;; ++r) {
        if (r >= cap && (r_U || r_F || r_maxmex || r_acc || r_seeds)) { status = ORC_EROUNDS; break; }
        /* compact the uncoloured list (the reference filters color == -1, coloring.py:86) */
        int64_t m = 0;
        for (int64_t i = 0; i < nunc; ++i) if (color[unc[i]] == -1) unc[m++] = unc[i];
        nunc = m;
        if (r_U) r_U[r] = nunc;
        if (r_F) r_F[r] = 0;
        if (r_maxmex) r_maxmex[r] = -1;
        if (r_acc) r_acc[r] = 0;
        if (r_seeds) r_seeds[r] = 0;
        sum->rounds = r + 1;
        if (nunc == 0) break;

        /* propose: colours as at the start of the round (broadcast, coloring.py:82-83) */
        int64_t nprop = 0, maxmex = -1, fails = 0;
        for (int64_t i = 0; i < nunc; ++i) {
            int64_t v = unc[i];
            ++stampc;
            int64_t ncol = 0;
            for (int64_t e = rp[v]; e < rp[v + 1]; ++e) {
                int32_t c = color[col[e]];
                if (c >= 0) { ncol++; if (c <= n) stamp[c] = stampc; }
            }
            int64_t mex;
            if (ncol == 0) {
                if (variant == 0 && !speculative) continue;  /* (-2, node): coloring.py:48-49  */
                mex = 0;                             /* (0, info): coloring_optimized.py:159-160;
                                                        speculative first-fit: everyone proposes */
                if (speculative && k >= 0 && mex >= k) fails++;
            } else {
                mex = 0;
                while (stamp[mex] == stampc) ++mex;
                if (k >= 0 && mex >= k) fails++;     /* (-3, node): coloring.py:53             */
            }
            cand[v] = mex;
            props[nprop++] = v;
            if (mex > maxmex) maxmex = mex;
            double d = (double)deg_of(rp, v);
            sum->balg_propose += 24.0 + 8.0 * d;
            sum->balg_resolve += 24.0 + 12.0 * d;
        }
        if (r_F) r_F[r] = nprop;
        if (r_maxmex) r_maxmex[r] = maxmex;
        if (fails > 0) {                             /* coloring.py:104-108 */
            status = ORC_FAILED;
            sum->fail_round = r;
            sum->fail_count = fails;
            break;
        }
        if (nprop == 0) {                            /* stall: coloring.py:93-95 spins */
            if (!e1) { status = ORC_STALLED; break; }
            int64_t seeds = e1_reseed(rp, col, n, color, colored_round, r + 1, parent, best);
            sum->reseeds += seeds;
            if (r_seeds) r_seeds[r] = seeds;
            for (int64_t i = 0; i < nunc; ++i) {
                int64_t v = unc[i];
                if (color[v] == 0) sum->balg_push += 16.0 + 8.0 * (double)deg_of(rp, v);
            }
            continue;
        }

        int64_t nacc = 0;
        if (speculative) {
            /* speculative first-fit, one-shot resolution (Luby / Jones-Plassmann depth 1):
               v keeps its proposal iff no LISTED neighbour of lower rank proposed the same
               colour this round; every other proposer retries next round */
            for (int64_t i = 0; i < nprop; ++i) acc_stamp[props[i]] = -3 - r;  /* proposer mark */
            for (int64_t i = 0; i < nprop; ++i) {
                int64_t v = props[i];
                int ok = 1;
                for (int64_t e = rp[v]; e < rp[v + 1] && ok; ++e) {
                    int64_t u = col[e];
                    if (u != v && (acc_stamp[u] == -3 - r || acc_stamp[u] == r) && cand[u] == cand[v] && rank_lt(u, v))
                        ok = 0;
                }
                if (ok) acc_stamp[v] = r;
            }
        } else if (variant == 0) {
            /* LFMIS per candidate colour under rank (deg asc, pos asc).  Groups are
               independent, so one pass in global rank order is the same computation. */
            qsort(props, (size_t)nprop, sizeof(int64_t), cmp_rank);
            for (int64_t i = 0; i < nprop; ++i) {
                int64_t v = props[i];
                int ok = 1;
                for (int64_t e = rp[v]; e < rp[v + 1]; ++e) {
                    int64_t u = col[e];
                    if (acc_stamp[u] == r && cand[u] == cand[v]) { ok = 0; break; }  /* LFMIS */
                }
                if (ok) acc_stamp[v] = r;
            }
        } else {
            /* arrival-order fold (file order; props inherits unc's increasing order),
               admit / evict rule */
            for (int64_t i = 0; i < nprop; ++i) {
                int64_t v = props[i];
                int64_t dv = deg_of(rp, v);
                int ok = 1;
                for (int64_t e = rp[v]; e < rp[v + 1]; ++e) {
                    int64_t u = col[e];
                    if (u != v && acc_stamp[u] == r && cand[u] == cand[v] && deg_of(rp, u) >= dv) { ok = 0; break; }
                }
                if (!ok) continue;
                acc_stamp[v] = r;
                /* evict admitted x of the group with v in N(x) and deg(x) < deg(v):
                   x ranges over v's in-neighbours (transpose) */
                for (int64_t e = trp[v]; e < trp[v + 1]; ++e) {
                    int64_t x = tcol[e];
                    if (acc_stamp[x] == r && cand[x] == cand[v] && deg_of(rp, x) < dv) acc_stamp[x] = -2 - r;
                }
            }
        }
        /* commit (coloring.py:117-127) */
        for (int64_t i = 0; i < nprop; ++i) {
            int64_t v = props[i];
            if (acc_stamp[v] == r) {
                color[v] = (int32_t)cand[v];
                if (colored_round) colored_round[v] = (int32_t)(r + 1);
                nacc++;
                sum->balg_push += 16.0 + 8.0 * (double)deg_of(rp, v);
            }
        }
        if (r_acc) r_acc[r] = nacc;
    }
    {
        int64_t mc = -1;
        for (int64_t v = 0; v < n; ++v) if (color[v] > mc) mc = color[v];
        sum->max_color = mc;
        sum->balg_validate = 20.0 * (double)n + 8.0 * (double)rp[n];
    }
out:
    free(cand); free(stamp); free(acc_stamp); free(props); free(unc); free(parent); free(best);
    free(trp); free(tcol);
    return status;
}

int oracle_color(const int64_t* rp, const int32_t* col, int64_t n, int32_t variant, int64_t k,
                 int32_t e1, int32_t* color, int32_t* colored_round,
                 int64_t* r_U, int64_t* r_F, int64_t* r_maxmex, int64_t* r_acc, int64_t* r_seeds,
                 int64_t cap, orc_summary* sum) {
    return color_impl(rp, col, n, variant, k, e1, NULL, 0, color, colored_round, r_U, r_F, r_maxmex, r_acc,
                      r_seeds, cap, sum);
}

/* Variant A with seeded priorities (priority = 1: rank = (prio_hash(seed, v), pos) replaces
   (deg, pos) in the per-colour LFMIS of coloring.py:56-70; the seed / E1 rule stays
   argmax (deg, pos)) and/or speculative first-fit rounds (speculative = 1: every
   uncoloured vertex proposes, one-shot resolution under the same rank). */
int oracle_color_prio(const int64_t* rp, const int32_t* col, int64_t n, int64_t k, int32_t e1, int32_t priority,
                      uint64_t seed, int32_t speculative, int32_t* color, int32_t* colored_round, int64_t* r_U,
                      int64_t* r_F, int64_t* r_maxmex, int64_t* r_acc, int64_t* r_seeds, int64_t cap,
                      orc_summary* sum) {
    uint32_t* key = NULL;
    if (priority) {
        key = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(n > 0 ? n : 1));
        if (!key) return ORC_ENOMEM;
        for (int64_t v = 0; v < n; ++v) key[v] = prio_hash(seed, v);
    }
    int st = color_impl(rp, col, n, 0, k, e1, key, speculative, color, colored_round, r_U, r_F, r_maxmex, r_acc,
                        r_seeds, cap, sum);
    free(key);
    return st;
}

/* validate_graph_coloring (coloring.py:149-162): uncoloured count and the directed
   count of listed pairs (v, u in N(v)) with colour[u] == colour[v]. */
void oracle_validate(const int64_t* rp, const int32_t* col, int64_t n, const int32_t* color,
                     int64_t* uncolored, int64_t* conflicts) {
    int64_t unc = 0, conf = 0;
    for (int64_t v = 0; v < n; ++v) {
        if (color[v] == -1) unc++;
        for (int64_t e = rp[v]; e < rp[v + 1]; ++e)
            if (color[col[e]] == color[v]) conf++;
    }
    *uncolored = unc;
    *conflicts = conf;
}
