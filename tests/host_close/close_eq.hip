// The round close two ways on the CPU (tests/test_host_close.py): gc_close_interleaved (the
// form rounds 1-3 run) and gc_close_batched with its words loaded first (GC_CLOSE_BATCH) must
// leave the same control block and the same round records for every mode and state.
//   close_eq TRIALS SEED   -> "ok TRIALS" or the first difference, exit 1
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "gc_close.h"

namespace {

constexpr int kRecs = 64;

struct Case {
    DevCtl c;
    std::vector<RoundRec> rec;
};

long long pick(std::mt19937_64& r, std::initializer_list<long long> special, long long lo, long long hi) {
    if (r() % 3 == 0) {
        auto it = special.begin();
        std::advance(it, (long)(r() % special.size()));
        return *it;
    }
    return lo + (long long)(r() % (unsigned long long)(hi - lo + 1));
}

}  // namespace

int main(int argc, char** argv) {
    const long long trials = argc > 1 ? atoll(argv[1]) : 100000;
    std::mt19937_64 r(argc > 2 ? strtoull(argv[2], nullptr, 10) : 1);
    for (long long t = 0; t < trials; ++t) {
        Case a;
        a.rec.resize(kRecs);
        // every byte random first: fields the close does not touch must survive both forms alike
        unsigned char* b = reinterpret_cast<unsigned char*>(&a.c);
        for (size_t i = 0; i < sizeof(DevCtl); ++i) b[i] = (unsigned char)r();
        unsigned char* rb = reinterpret_cast<unsigned char*>(a.rec.data());
        for (size_t i = 0; i < sizeof(RoundRec) * kRecs; ++i) rb[i] = (unsigned char)r();
        DevCtl& c = a.c;
        const long long n = pick(r, {1, 64, 4096}, 1, 1 << 20);
        c.halt = (int)pick(r, {0, 0, 0, GC_H_SWEEPS}, 0, 9);
        c.cur = (int)(r() & 1);
        c.e1 = (int)(r() & 1);
        c.fcnt[0] = (ull)pick(r, {0, (n + 63) / 64, n / 64, 1}, 0, n);
        c.fcnt[1] = (ull)pick(r, {0, (n + 63) / 64, n / 64, 1}, 0, n);
        c.seedkey = (ull)pick(r, {0}, 0, 1ll << 40);
        c.U = pick(r, {0, 1, n}, 0, n);
        c.sweeps = pick(r, {0, 1, 2}, 0, 40);
        c.sweep_total = pick(r, {0}, 0, 1 << 20);
        c.maxdepth = pick(r, {0, c.sweeps, c.sweeps + 1}, 0, 40);
        c.bigsweeps = pick(r, {0}, 0, 40);
        c.hugesweeps = pick(r, {0}, 0, 40);
        c.maxmex = pick(r, {-1, 0, 61, 62}, -1, 5000);
        c.rbase = pick(r, {0}, 0, 1 << 20);
        c.round = c.rbase + pick(r, {0, kRecs - 6, kRecs - 5, kRecs - 4, kRecs - 3}, 0, kRecs - 3);
        c.rcap = kRecs;
        const int mode = (int)pick(r, {GC_CM_ROUND, GC_CM_ROUND}, GC_CM_ROUND, GC_CM_RESEED);
        const int allow_big = (int)(r() & 1), fused = (int)(r() & 1);
        GcClosePre pre;
        pre.accepted = (ull)pick(r, {0, (long long)c.U}, 0, c.U);
        pre.nx_failcnt = (ull)pick(r, {0}, 0, 100);
        pre.nx_maxmex = pick(r, {-1, 0}, -1, 5000);
        pre.uncolored = (ull)pick(r, {0, 1}, 0, n);
        pre.fnext = (ull)pick(r, {0, 0, 1}, 0, n);
        Case x = a;  // the batched form's copy
        GDev g{};
        g.n = n;
        GLists L{};
        L.rec = a.rec.data();
        gc_close_interleaved(g, L, &a.c, mode, allow_big, fused, pre);
        GLists Lx{};
        Lx.rec = x.rec.data();
        const GcCloseCtl k = gc_close_load(&x.c);
        gc_close_batched(g, Lx, &x.c, mode, allow_big, fused, pre, k);
        if (memcmp(&a.c, &x.c, sizeof(DevCtl)) != 0 || memcmp(a.rec.data(), x.rec.data(), sizeof(RoundRec) * kRecs) != 0) {
            const unsigned char* p = reinterpret_cast<const unsigned char*>(&a.c);
            const unsigned char* q = reinterpret_cast<const unsigned char*>(&x.c);
            size_t off = 0;
            while (off < sizeof(DevCtl) && p[off] == q[off]) ++off;
            printf("trial %lld: mode %d allow_big %d fused %d: first difference at control byte %zu%s\n", t, mode,
                   allow_big, fused, off, off == sizeof(DevCtl) ? " (records differ)" : "");
            return 1;
        }
    }
    printf("ok %lld\n", trials);
    return 0;
}
