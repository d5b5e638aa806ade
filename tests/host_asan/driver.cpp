// Host-side sanitizer driver (TEST INFRASTRUCTURE): the native file readers and writers of
// csrc/gc_io_host.cpp and the generator of csrc/gc_gen_host.cpp, built with
// -fsanitize=address,undefined by tests/test_host_asan.py (the host code is
// the part of the drop-in that reads untrusted files).  No GPU code is involved.
//   driver read  FILE...            gc_json_read_graph on each file: "<status> <n> <nnz> <sum>"
//   driver csr   FILE...            gc_csr_read on each file: the same line
//   driver write DIR                every writer on a generated graph, then re-reads what it wrote
//   driver gen   N D SEED           gc_gen_uniform: "<status> <nnz> <sum>"
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "gcolor.h"

// gc_set_error / gc_last_error live in the HIP part of libgcolor.so; the driver links only
// the host sources, so it carries its own (same contract: a thread-local message)
static thread_local std::string g_err;
void gc_set_error(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}
extern "C" const char* gc_last_error(void) { return g_err.c_str(); }

static unsigned long long checksum(const gc_csr* c) {
    unsigned long long s = 1469598103934665603ull;
    for (int64_t i = 0; i <= c->n; ++i) s = (s ^ (unsigned long long)c->row_ptr[i]) * 1099511628211ull;
    for (int64_t i = 0; i < c->nnz; ++i) s = (s ^ (unsigned long long)(unsigned)c->col[i]) * 1099511628211ull;
    if (c->ids)
        for (int64_t i = 0; i < c->n; ++i) s = (s ^ (unsigned long long)c->ids[i]) * 1099511628211ull;
    return s;
}

static void report(int st, gc_csr* c) {
    if (st == GC_OK && c) {
        printf("%d %lld %lld %llu\n", st, (long long)c->n, (long long)c->nnz, checksum(c));
        gc_csr_free(c);
    } else {
        printf("%d 0 0 0\n", st);
    }
}

int main(int argc, char** argv) {
    setvbuf(stdout, nullptr, _IOLBF, 0);
    if (argc < 2) return 2;
    const std::string mode = argv[1];
    if (mode == "read" || mode == "csr") {
        for (int i = 2; i < argc; ++i) {
            gc_csr* c = nullptr;
            const int st = mode == "read" ? gc_json_read_graph(argv[i], &c) : gc_csr_read(argv[i], &c);
            report(st, c);
        }
        return 0;
    }
    if (mode == "gen" && argc == 5) {
        const int64_t n = atoll(argv[2]);
        const int D = atoi(argv[3]);
        const uint64_t seed = strtoull(argv[4], nullptr, 10);
        std::vector<int64_t> rp((size_t)n + 1);
        std::vector<int32_t> col((size_t)(n * D + 1));
        int64_t nnz = 0;
        const int st = gc_gen_uniform(n, D, seed, rp.data(), col.data(), (int64_t)col.size(), &nnz);
        unsigned long long s = 0;
        for (int64_t i = 0; i < nnz; ++i) s = s * 31 + (unsigned)col[(size_t)i];
        printf("%d %lld %llu\n", st, (long long)nnz, s);
        return 0;
    }
    if (mode == "write" && argc == 3) {
        const std::string dir = argv[2];
        const int64_t n = 50;
        std::vector<int64_t> rp((size_t)n + 1), ids((size_t)n);
        std::vector<int32_t> col, colors((size_t)n);
        rp[0] = 0;
        for (int64_t v = 0; v < n; ++v) {
            for (int64_t d = 1; d <= v % 4; ++d) col.push_back((int32_t)((v + d * 7) % n));
            rp[(size_t)v + 1] = (int64_t)col.size();
            ids[(size_t)v] = v * 1000003 - 25;
            colors[(size_t)v] = (int32_t)(v % 5) - 1;
        }
        int st = gc_json_write_coloring((dir + "/c.json").c_str(), ids.data(), colors.data(), n);
        st |= gc_json_write_coloring((dir + "/c0.json").c_str(), nullptr, colors.data(), 0);
        st |= gc_json_write_graph((dir + "/g.json").c_str(), ids.data(), rp.data(), col.data(), n, colors.data());
        st |= gc_json_write_graph((dir + "/g2.json").c_str(), nullptr, rp.data(), col.data(), n, nullptr);
        st |= gc_csr_write((dir + "/g.gcsr").c_str(), rp.data(), col.data(), ids.data(), n, (int64_t)col.size(), 0);
        st |= gc_csr_write((dir + "/g2.gcsr").c_str(), rp.data(), col.data(), nullptr, n, (int64_t)col.size(), 1);
        printf("write %d\n", st);
        for (const char* f : {"/g.json", "/g2.json"}) {
            gc_csr* c = nullptr;
            const int rs = gc_json_read_graph((dir + f).c_str(), &c);
            report(rs, c);
        }
        for (const char* f : {"/g.gcsr", "/g2.gcsr"}) {
            gc_csr* c = nullptr;
            const int rs = gc_csr_read((dir + f).c_str(), &c);
            report(rs, c);
        }
        return 0;
    }
    return 2;
}
