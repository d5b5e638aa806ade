// gc_gen_host.cpp -- native version of the reference generator's process (graph.py:30-43).
//
// For each node in id order: target = U{0..D}; while deg(node) < target, draw a random
// partner, keep it iff it is not the node itself, not already adjacent and below D.
// Symmetric, simple, max degree <= D, adjacency kept in insertion order (as Node.neighbors).
// The random stream is splitmix64 (not Python's MT19937): same process, different
// draws; small graphs that must match the reference bit-for-bit go through the Python
// generator (gcolor_amd.generators.reference_graph) instead.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "gcolor.h"

void gc_set_error(const char* fmt, ...);

namespace {
struct SplitMix {
    uint64_t s;
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    uint64_t below(uint64_t n) { return (uint64_t)(((unsigned __int128)next() * n) >> 64); }
};
}  // namespace

extern "C" int gc_gen_uniform(int64_t n, int32_t D, uint64_t seed, int64_t* row_ptr, int32_t* col, int64_t col_cap,
                              int64_t* nnz_out) {
    if (n < 0 || n >= (1ll << 31) - 1 || D < 0 || !row_ptr || !nnz_out) {
        gc_set_error("gc_gen_uniform: invalid arguments");
        return GC_EINVAL;
    }
    std::vector<int32_t> slots((size_t)n * (size_t)D);
    std::vector<int32_t> deg((size_t)n, 0);
    SplitMix rng{seed};
    for (int64_t v = 0; v < n; ++v) {
        const int32_t target = (int32_t)rng.below((uint64_t)D + 1);
        int64_t rejects = 0;
        while (deg[v] < target) {
            const int64_t u = (int64_t)rng.below((uint64_t)n);
            bool ok = u != v && deg[u] < D;
            if (ok) {
                const int32_t* nb = &slots[(size_t)v * D];
                for (int32_t i = 0; i < deg[v]; ++i)
                    if (nb[i] == u) { ok = false; break; }
            }
            if (ok) {
                slots[(size_t)v * D + deg[v]++] = (int32_t)u;
                slots[(size_t)u * D + deg[u]++] = (int32_t)v;
                rejects = 0;
                continue;
            }
            // the reference spins forever when no admissible partner exists.
            if (++rejects > 64ll * (D + 1) + 4096) {
                bool any = false;
                for (int64_t w = 0; w < n && !any; ++w) {
                    if (w == v || deg[w] >= D) continue;
                    bool adj = false;
                    for (int32_t i = 0; i < deg[v]; ++i)
                        if (slots[(size_t)v * D + i] == w) { adj = true; break; }
                    any = !adj;
                }
                if (!any) break;
                rejects = 0;
            }
        }
    }
    int64_t e = 0;
    row_ptr[0] = 0;
    for (int64_t v = 0; v < n; ++v) {
        if (col) {
            if (e + deg[v] > col_cap) { gc_set_error("gc_gen_uniform: col capacity too small"); return GC_EINVAL; }
            memcpy(col + e, &slots[(size_t)v * D], sizeof(int32_t) * (size_t)deg[v]);
        }
        e += deg[v];
        row_ptr[v + 1] = e;
    }
    *nnz_out = e;
    return GC_OK;
}
