/* The CPU oracles under AddressSanitizer + UndefinedBehaviorSanitizer (TEST INFRASTRUCTURE):
   oracle/gcolor_oracle.c (variants A and B, bounded k, E1 on / off, seeded priorities, the
   speculative mode) and oracle/gcolor_omp.c (OpenMP) on seeded random directed multigraphs
   with self-loops, isolated vertices and hubs; every run is cross-checked (the OpenMP
   restatement against the single-thread oracle, colours and per-round records).  A sanitizer
   report or a mismatch exits non-zero.  Built and run by tests/test_host_asan.py. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int64_t rounds, fail_round, fail_count, reseeds, max_color;
    double balg_propose, balg_resolve, balg_push, balg_validate;
} orc_summary;
int oracle_color(const int64_t* rp, const int32_t* col, int64_t n, int32_t variant, int64_t k, int32_t e1,
                 int32_t* color, int32_t* colored_round, int64_t* r_U, int64_t* r_F, int64_t* r_maxmex,
                 int64_t* r_acc, int64_t* r_seeds, int64_t cap, orc_summary* sum);
int oracle_color_prio(const int64_t* rp, const int32_t* col, int64_t n, int64_t k, int32_t e1, int32_t priority,
                      uint64_t seed, int32_t speculative, int32_t* color, int32_t* colored_round, int64_t* r_U,
                      int64_t* r_F, int64_t* r_maxmex, int64_t* r_acc, int64_t* r_seeds, int64_t cap,
                      orc_summary* sum);
int omp_color(const int64_t* rp, const int32_t* col, int64_t n, int32_t symmetric, int32_t nthreads,
              int32_t* color, int32_t* colored_round, int64_t* r_U, int64_t* r_F, int64_t* r_maxmex,
              int64_t* r_acc, int64_t* r_seeds, int64_t cap, int64_t* rounds_out, int64_t* reseeds_out);

static uint64_t rs = 88172645463325252ull;
static uint64_t rnd(void) { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return rs; }

#define CAP 100000

int main(int argc, char** argv) {
    const int graphs = argc > 1 ? atoi(argv[1]) : 40;
    int64_t* rec[10];
    for (int i = 0; i < 10; ++i) rec[i] = (int64_t*)calloc(CAP, sizeof(int64_t));
    for (int t = 0; t < graphs; ++t) {
        const int64_t n = (int64_t)(rnd() % 400);
        const int64_t m = n ? (int64_t)(rnd() % (6 * (uint64_t)n + 1)) : 0;
        const int sym = (int)(t % 2);
        int64_t* deg = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
        int32_t* src = (int32_t*)malloc(sizeof(int32_t) * (size_t)(2 * m + 1));
        int32_t* dst = (int32_t*)malloc(sizeof(int32_t) * (size_t)(2 * m + 1));
        int64_t e = 0;
        for (int64_t i = 0; i < m; ++i) {
            /* a few hubs: vertex 0 and 1 take many edges */
            const int32_t a = (int32_t)((rnd() % 4 == 0) ? rnd() % 2 : rnd() % (uint64_t)n);
            const int32_t b = (int32_t)(rnd() % (uint64_t)n);
            if (sym && a == b) continue;
            src[e] = a; dst[e] = b; ++e;
            if (sym) { src[e] = b; dst[e] = a; ++e; }
        }
        for (int64_t i = 0; i < e; ++i) deg[src[i] + 1]++;
        for (int64_t v = 0; v < n; ++v) deg[v + 1] += deg[v];
        int32_t* col = (int32_t*)malloc(sizeof(int32_t) * (size_t)(e + 1));
        int64_t* pos = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 1));
        memcpy(pos, deg, sizeof(int64_t) * (size_t)(n + 1));
        for (int64_t i = 0; i < e; ++i) col[pos[src[i]]++] = dst[i];
        int32_t* c1 = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1));
        int32_t* r1 = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1));
        int32_t* c2 = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1));
        int32_t* r2 = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1));
        orc_summary s;
        for (int variant = 0; variant < 2; ++variant)
            for (int64_t k = -1; k < 3; ++k)
                for (int e1 = 0; e1 < 2; ++e1) {
                    int st = oracle_color(deg, col, n, variant, k, e1, c1, r1, rec[0], rec[1], rec[2], rec[3], rec[4],
                                          CAP, &s);
                    if (st < 0) { fprintf(stderr, "oracle_color status %d\n", st); return 1; }
                }
        for (int prio = 0; prio < 2; ++prio)
            for (int spec = 0; spec < 2; ++spec) {
                int st = oracle_color_prio(deg, col, n, -1, 1, prio, 12345u + (uint64_t)t, spec, c1, r1, rec[0], rec[1],
                                           rec[2], rec[3], rec[4], CAP, &s);
                if (st < 0) { fprintf(stderr, "oracle_color_prio status %d\n", st); return 1; }
            }
        /* the OpenMP restatement against the oracle: variant A, unbounded, E1 on */
        int st = oracle_color(deg, col, n, 0, -1, 1, c1, r1, rec[0], rec[1], rec[2], rec[3], rec[4], CAP, &s);
        int64_t rounds = 0, reseeds = 0;
        int st2 = omp_color(deg, col, n, sym, 1 + t % 4, c2, r2, rec[5], rec[6], rec[7], rec[8], rec[9], CAP, &rounds,
                            &reseeds);
        if (st < 0 || st2 < 0 || rounds != s.rounds || reseeds != s.reseeds ||
            memcmp(c1, c2, sizeof(int32_t) * (size_t)n) || memcmp(r1, r2, sizeof(int32_t) * (size_t)n)) {
            fprintf(stderr, "graph %d: omp_color differs from oracle_color (status %d/%d rounds %lld/%lld)\n", t, st,
                    st2, (long long)s.rounds, (long long)rounds);
            return 1;
        }
        for (int i = 0; i < 5; ++i)
            if (memcmp(rec[i], rec[5 + i], sizeof(int64_t) * (size_t)rounds)) {
                fprintf(stderr, "graph %d: per-round record %d differs\n", t, i);
                return 1;
            }
        free(deg); free(src); free(dst); free(col); free(pos); free(c1); free(r1); free(c2); free(r2);
    }
    for (int i = 0; i < 10; ++i) free(rec[i]);
    printf("ok %d graphs\n", graphs);
    return 0;
}
