// gc_graph.hip -- device CSR construction: host/device CSR import, in-neighbour
// transpose, and the synthetic generators of BASELINE.md (R-MAT, 3-D 7-point mesh).
//
// Replaces the reference's data model (Node objects with linked neighbours,
// node.py:1-18, graph.py:15-28) and its RDD distribution (coloring.py:201-209): the
// graph becomes three HBM-resident arrays (rp int64[n+1], col int32[nnz], deg int32[n]).
#include <cstring>
#include <string.h>

#include <rocprim/rocprim.hpp>

#include <algorithm>

#include "gc_engine.h"

// ------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------
// in-neighbour CSR of the rows [lo, hi): for every target u, the rows in range listing u
__global__ void k_count_targets(const long long* rp, const int* col, long long lo, long long hi, ull* cnt) {
    for (long long v = lo + (long long)blockIdx.x * blockDim.x + threadIdx.x; v < hi; v += (long long)gridDim.x * blockDim.x)
        for (long long e = rp[v]; e < rp[v + 1]; ++e) atomicAdd(&cnt[col[e]], 1ull);
}

__global__ void k_fill_transpose(const long long* rp, const int* col, long long lo, long long hi, const long long* trp,
                                 ull* cursor, int* tcol) {
    for (long long v = lo + (long long)blockIdx.x * blockDim.x + threadIdx.x; v < hi; v += (long long)gridDim.x * blockDim.x)
        for (long long e = rp[v]; e < rp[v + 1]; ++e) {
            const int u = col[e];
            const ull p = atomicAdd(&cursor[u], 1ull);
            tcol[trp[u] + (long long)p] = (int)v;
        }
}

// The same for a SYMMETRIC graph, without atomics: the rows in [lo, hi) that list u are
// the entries of u's own row that fall in [lo, hi).  A wave per row (a hub's row is walked
// by 64 lanes: one thread per row walked R-MAT-24's 4e5-entry hub rows serially, 1.4 s of
// shard set-up), entries kept in row order by ballot compaction.
__global__ void k_filter_count(const long long* rp, const int* col, long long n, long long lo, long long hi,
                               long long* cnt) {
    const int lane = gc_lane();
    const long long waves = (long long)gridDim.x * (blockDim.x / GC_WAVE);
    for (long long v = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / GC_WAVE; v < n; v += waves) {
        long long c = 0;
        for (long long e = rp[v] + lane; e < rp[v + 1]; e += GC_WAVE) c += (col[e] >= lo && col[e] < hi) ? 1 : 0;
        c = gc_wave_sum(c);
        if (lane == 0) cnt[v] = c;
    }
}

__global__ void k_filter_fill(const long long* rp, const int* col, long long n, long long lo, long long hi,
                              const long long* trp, int* tcol) {
    const int lane = gc_lane();
    const long long waves = (long long)gridDim.x * (blockDim.x / GC_WAVE);
    for (long long v = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / GC_WAVE; v < n; v += waves) {
        long long base = trp[v];
        const long long e1 = rp[v + 1];
        for (long long e0 = rp[v]; e0 < e1; e0 += GC_WAVE) {
            const long long e = e0 + lane;
            const int u = e < e1 ? col[e] : -1;
            const bool keep = u >= lo && u < hi;
            const ull m = __ballot(keep);
            if (keep) tcol[base + __popcll(m & gc_lanemask_lt())] = u;
            base += __popcll(m);
        }
    }
}

// R-MAT edge generator.  Counter-based RNG (splitmix64 of seed, edge index, level pair)
// so the graph is a pure function of (scale, edge_factor, a, b, c, seed).
__device__ __forceinline__ ull gc_splitmix(ull x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void k_rmat_edges(long long m, int scale, double a, double b, double c, ull seed, ull* keys) {
    const unsigned ta = (unsigned)(a * 4294967296.0);
    const unsigned tb = (unsigned)((a + b) * 4294967296.0);
    const unsigned tc = (unsigned)((a + b + c) * 4294967296.0);
    const ull sentinel = (scale * 2 == 64) ? ~0ull : ((1ull << (2 * scale)) - 1ull);
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (long long)gridDim.x * blockDim.x) {
        ull src = 0, dst = 0;
        ull h = 0;
        for (int lvl = 0; lvl < scale; ++lvl) {
            if ((lvl & 1) == 0) h = gc_splitmix(seed ^ gc_splitmix((ull)i * 64ull + (ull)(lvl >> 1)));
            const unsigned r = (lvl & 1) ? (unsigned)(h >> 32) : (unsigned)h;
            const unsigned q = r < ta ? 0u : (r < tb ? 1u : (r < tc ? 2u : 3u));
            src = (src << 1) | (q >> 1);
            dst = (dst << 1) | (q & 1u);
        }
        if (src == dst) {
            keys[2 * i] = sentinel;
            keys[2 * i + 1] = sentinel;
        } else {
            keys[2 * i] = (src << scale) | dst;
            keys[2 * i + 1] = (dst << scale) | src;
        }
    }
}

__global__ void k_keys_to_csr(const ull* keys, long long m, int scale, int* col) {
    const ull mask = (1ull << scale) - 1ull;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (long long)gridDim.x * blockDim.x)
        col[i] = (int)(keys[i] & mask);
}

// rp[v] = lower_bound(keys, v << scale)
__global__ void k_row_bounds(const ull* keys, long long m, int scale, long long n, long long* rp) {
    for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v <= n; v += (long long)gridDim.x * blockDim.x) {
        const ull needle = (ull)v << scale;
        long long lo = 0, hi = m;
        while (lo < hi) {
            const long long mid = lo + ((hi - lo) >> 1);
            if (keys[mid] < needle) lo = mid + 1;
            else hi = mid;
        }
        rp[v] = (v == n) ? m : lo;
    }
}

__global__ void k_mesh_deg(long long nx, long long ny, long long nz, long long* cnt) {
    const long long n = nx * ny * nz;
    for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (long long)gridDim.x * blockDim.x) {
        const long long x = v % nx, y = (v / nx) % ny, z = v / (nx * ny);
        cnt[v] = (x > 0) + (x < nx - 1) + (y > 0) + (y < ny - 1) + (z > 0) + (z < nz - 1);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) cnt[n] = 0;
}

__global__ void k_mesh_fill(long long nx, long long ny, long long nz, const long long* rp, int* col) {
    const long long n = nx * ny * nz;
    for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (long long)gridDim.x * blockDim.x) {
        const long long x = v % nx, y = (v / nx) % ny, z = v / (nx * ny);
        long long e = rp[v];
        if (x > 0) col[e++] = (int)(v - 1);
        if (x < nx - 1) col[e++] = (int)(v + 1);
        if (y > 0) col[e++] = (int)(v - nx);
        if (y < ny - 1) col[e++] = (int)(v + nx);
        if (z > 0) col[e++] = (int)(v - nx * ny);
        if (z < nz - 1) col[e++] = (int)(v + nx * ny);
    }
}

// ------------------------------------------------------------------------------------
// host helpers
// ------------------------------------------------------------------------------------
static int grid_for(long long items, int cap = 8192) {
    long long b = (items + GC_BLOCK - 1) / GC_BLOCK;
    return (int)std::max<long long>(1, std::min<long long>(b, cap));
}

static int exclusive_scan_ll(const long long* in, long long* out, long long count, hipStream_t s) {
    size_t bytes = 0;
    GC_HIP(rocprim::exclusive_scan(nullptr, bytes, in, out, 0ll, (size_t)count, rocprim::plus<long long>(), s));
    void* tmp = nullptr;
    GC_HIP(gc_dmalloc(&tmp, bytes ? bytes : 1));
    hipError_t e = rocprim::exclusive_scan(tmp, bytes, in, out, 0ll, (size_t)count, rocprim::plus<long long>(), s);
    const hipError_t se = hipStreamSynchronize(s);
    gc_dfree(tmp);
    GC_HIP(e);
    GC_HIP(se);
    return GC_OK;
}

void gc_free_all(gc_graph* g) {
    if (!g) return;
    hipSetDevice(g->device);
    if (g->stream) hipStreamSynchronize(g->stream);  // parked blocks are idle (gc_alloc.hip)
    {
        void* prep[] = {g->kb, g->tile_r0, g->seg_row, g->seg_j, g->seg_aux, g->seg_cls, g->seg_base, g->hubmap, g->hubflag};
        for (void* p : prep)
            if (p) gc_dfree(p);
    }
    if (g->trp && g->trp != g->rp) gc_dfree(g->trp);
    if (g->tcol && g->tcol != g->col) gc_dfree(g->tcol);
    gc_hubs_free(g);
    if (g->borrowed) {  // a shard's view: the CSR belongs to the replicated graph handle
        g->rp = nullptr;
        g->col = nullptr;
        g->deg = nullptr;
        g->nlow = nullptr;
    }
    void* ptrs[] = {g->rp, g->col, g->deg, g->color, g->cround, g->cand, g->c8, g->c4, g->k8, g->nlow, g->inF, g->mark, g->F[0],
                    g->F[1], g->heavy, g->wide, g->undL[0], g->undL[1], g->undL[2], g->undH[0], g->undH[1],
                    g->undH[2], g->seeds[0], g->seeds[1], g->ulist, g->parent, g->best, g->vcolors, g->lcur, g->neq, g->nhe, g->bpend, g->bwatch, g->hpl, g->hplc, g->bstat, g->accs, g->bigw, g->rec, g->fsum, g->ctl};
    for (void* p : ptrs)
        if (p) gc_dfree(p);
    if (g->hctl) gc_dfree(g->hctl);
    if (g->hsnap) gc_dfree(g->hsnap);
    for (auto e : g->evsnap)
        if (e) hipEventDestroy(e);
    for (auto e : g->evpool) hipEventDestroy(e);
    if (g->ev0) hipEventDestroy(g->ev0);
    if (g->ev1) hipEventDestroy(g->ev1);
    if (g->stream && g->own_stream) hipStreamDestroy(g->stream);
}

static int new_graph(gc_graph** out, long long n, long long nnz, uint32_t flags, gc_graph** res) {
    *res = nullptr;
    if (!out) { gc_set_error("null output handle"); return GC_EINVAL; }
    if (n < 0 || n >= (1ll << 31) - 1 || nnz < 0) {
        gc_set_error("unsupported graph size n=%lld nnz=%lld (positions are int32)", n, nnz);
        return GC_EINVAL;
    }
    gc_graph* g = new gc_graph();
    g->n = n;
    g->nnz = nnz;
    g->flags = flags;
    hipGetDevice(&g->device);
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipEventCreate(&g->ev0)) != hipSuccess || (e = hipEventCreate(&g->ev1)) != hipSuccess ||
        (e = gc_dmalloc((void**)&g->ctl, sizeof(DevCtl))) != hipSuccess ||
        (e = gc_hmalloc((void**)&g->hctl, sizeof(DevCtl))) != hipSuccess ||
        (e = gc_dmalloc((void**)&g->rp, sizeof(long long) * (size_t)(n + 1))) != hipSuccess ||
        (e = gc_dmalloc((void**)&g->col, sizeof(int) * (size_t)std::max<long long>(nnz, 1))) != hipSuccess ||
        (e = gc_dmalloc((void**)&g->deg, sizeof(int) * (size_t)std::max<long long>(n, 1))) != hipSuccess) {
        gc_set_error("graph allocation failed: %s", hipGetErrorString(e));
        gc_free_all(g);
        delete g;
        return GC_ENOMEM;
    }
    *res = g;
    return GC_OK;
}

// deg, kb, maxdeg and the rp checks; the rank partition of the input rows `src` (device,
// file order) into g->col (rows lower-rank first, coloring.py:64: see gc_prep.hip) with
// the column range check folded in; the transpose unless symmetric.
int gc_alloc_graph_common(gc_graph* g, const int* src) {
    hipStream_t s = g->stream;
    const size_t n1 = (size_t)std::max<long long>(g->n, 1);
    GC_HIP(gc_dmalloc((void**)&g->nlow, sizeof(int) * n1));
    GC_HIP(gc_dmalloc((void**)&g->neq, sizeof(int) * n1));
    GC_HIP(gc_dmalloc((void**)&g->nhe, sizeof(int) * n1));
    GC_HIP(gc_dmalloc((void**)&g->kb, n1));
    GC_HIP(hipMemsetAsync(g->ctl, 0, sizeof(DevCtl), s));
    if (g->n > 0)
        gcl_degrees(g->rp, (int)g->n, g->nnz, g->deg, g->kb, &g->ctl->seedkey, &g->ctl->list_cnt, grid_for(g->n), s);
    GC_HIP(hipGetLastError());
    GC_HIP(hipMemcpyAsync(g->hctl, g->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, s));
    GC_HIP(hipStreamSynchronize(s));
    if (g->hctl->list_cnt) {
        gc_set_error("row_ptr is not a CSR offset array (rp[0] != 0, rp[n] != nnz or decreasing)");
        return GC_EINVAL;
    }
    g->maxdeg = (long long)g->hctl->seedkey;
    if (g->maxdeg >= (1ll << 31)) { gc_set_error("degree too large"); return GC_EINVAL; }
    // symmetric graphs with hubs: the partition also marks the hub entries (a byte each), so
    // the hub transpose streams them instead of gathering a hub bit per entry (R-MAT-28: ~60 ms)
    const int hub_t = gc_hub_threshold();
    const bool flags_on = !(getenv("GC_HUB_FLAGS") && atoi(getenv("GC_HUB_FLAGS")) == 0);  // 0: A/B against the gathers
    if ((g->flags & GC_GRAPH_SYMMETRIC) && hub_t >= 0 && g->maxdeg > hub_t && g->nnz > 0 &&
        gc_partition_hubflags_supported() && flags_on) {
        if (gc_dmalloc((void**)&g->hubflag, (size_t)g->nnz) == hipSuccess) g->hubflag_t = hub_t;
        else g->hubflag = nullptr;  // no room: the transpose gathers instead
    }
    int rc = gc_partition(g, src, g->col, GC_PRIORITY_REF, 0, &g->ctl->conflicts, g->hubflag, g->hubflag_t);
    if (rc) return rc;
    GC_HIP(hipMemcpyAsync(g->hctl, g->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, s));
    GC_HIP(hipStreamSynchronize(s));
    if (g->hctl->conflicts) {
        gc_set_error("%llu adjacency entries are outside [0, n)", (unsigned long long)g->hctl->conflicts);
        return GC_EINVAL;
    }
    g->part_prio = GC_PRIORITY_REF;
    g->bpart = true;  // the reference partition splits every low part by degree too (variant B)
    if (g->flags & GC_GRAPH_SYMMETRIC) {
        g->trp = g->rp;
        g->tcol = g->col;
        return GC_OK;
    }
    // in-neighbour CSR for the frontier push (directed semantics of listed adjacency)
    return gc_build_in_csr(g, 0, g->n);
}

// In-neighbour CSR of the rows [lo, hi) into g->trp / g->tcol: for every vertex u, the
// rows in [lo, hi) that list u.  [0, n) is the full transpose; a shard builds the part
// its own rows contribute (gc_shard.hip).
int gc_build_in_csr(gc_graph* g, long long lo, long long hi) {
    hipStream_t s = g->stream;
    long long e0 = 0, e1 = 0;
    GC_READ(s, &e0, g->rp + lo, 1);
    GC_READ(s, &e1, g->rp + hi, 1);
    long long* cnt = nullptr;
    GC_HIP(gc_dmalloc((void**)&cnt, sizeof(long long) * (size_t)(g->n + 1)));
    GC_HIP(gc_dmalloc((void**)&g->trp, sizeof(long long) * (size_t)(g->n + 1)));
    GC_HIP(gc_dmalloc((void**)&g->tcol, sizeof(int) * (size_t)std::max<long long>(e1 - e0, 1)));
    GC_HIP(hipMemsetAsync(cnt, 0, sizeof(long long) * (size_t)(g->n + 1), s));
    if (hi > lo)
        hipLaunchKernelGGL(k_count_targets, dim3(grid_for(hi - lo)), dim3(GC_BLOCK), 0, s, g->rp, g->col, lo, hi,
                           (ull*)cnt);
    int rc = exclusive_scan_ll(cnt, g->trp, g->n + 1, s);
    if (rc) { gc_dfree(cnt); return rc; }
    GC_HIP(hipMemsetAsync(cnt, 0, sizeof(long long) * (size_t)(g->n + 1), s));
    if (hi > lo)
        hipLaunchKernelGGL(k_fill_transpose, dim3(grid_for(hi - lo)), dim3(GC_BLOCK), 0, s, g->rp, g->col, lo, hi,
                           g->trp, (ull*)cnt, g->tcol);
    GC_HIP(hipGetLastError());
    GC_HIP(hipStreamSynchronize(s));
    gc_dfree(cnt);
    return GC_OK;
}

// gc_build_in_csr for a symmetric graph (k_filter_*: no atomics)
int gc_build_in_csr_sym(gc_graph* g, long long lo, long long hi) {
    hipStream_t s = g->stream;
    long long* cnt = nullptr;
    GC_HIP(gc_dmalloc((void**)&cnt, sizeof(long long) * (size_t)(g->n + 1)));
    GC_HIP(gc_dmalloc((void**)&g->trp, sizeof(long long) * (size_t)(g->n + 1)));
    GC_HIP(hipMemsetAsync(cnt, 0, sizeof(long long) * (size_t)(g->n + 1), s));
    const int grid = gc_grid_for_waves(std::max<long long>(g->n, 1) * GC_WAVE, 8192);
    if (g->n > 0) hipLaunchKernelGGL(k_filter_count, dim3(grid), dim3(GC_BLOCK), 0, s, g->rp, g->col, g->n, lo, hi, cnt);
    int rc = exclusive_scan_ll(cnt, g->trp, g->n + 1, s);
    gc_dfree(cnt);
    if (rc) return rc;
    long long e = 0;
    GC_READ(s, &e, (const long long*)g->trp + g->n, 1);
    GC_HIP(gc_dmalloc((void**)&g->tcol, sizeof(int) * (size_t)std::max<long long>(e, 1)));
    if (g->n > 0)
        hipLaunchKernelGGL(k_filter_fill, dim3(grid), dim3(GC_BLOCK), 0, s, g->rp, g->col, g->n, lo, hi, g->trp, g->tcol);
    GC_HIP(hipGetLastError());
    GC_HIP(hipStreamSynchronize(s));
    return GC_OK;
}

// src: the input rows (device, file order); scratch: a library buffer holding them, freed here
static int finish_create(gc_graph* g, gc_graph** out, const int* src, int* scratch) {
    int rc = gc_alloc_graph_common(g, src);
    if (scratch) {
        hipStreamSynchronize(g->stream);
        gc_dfree(scratch);
    }
    if (rc) {
        std::string keep = gc_last_error();
        gc_free_all(g);
        delete g;
        gc_set_error("%s", keep.c_str());
        return rc;
    }
    *out = g;
    return GC_OK;
}

static int alloc_scratch(gc_graph* g, int** p) {
    if (gc_dmalloc((void**)p, sizeof(int) * (size_t)std::max<long long>(g->nnz, 1)) != hipSuccess) {
        gc_free_all(g);
        delete g;
        gc_set_error("allocation of the input rows (%lld entries) failed", g->nnz);
        return GC_ENOMEM;
    }
    return GC_OK;
}

extern "C" int gc_graph_create(const int64_t* row_ptr, const int32_t* col, int64_t n, int64_t nnz, uint32_t flags,
                               gc_graph** out) {
    if (!row_ptr || (nnz > 0 && !col)) { gc_set_error("gc_graph_create: null input"); return GC_EINVAL; }
    if (n < 0 || row_ptr[0] != 0 || row_ptr[n] != nnz) { gc_set_error("gc_graph_create: row_ptr[0] != 0 or row_ptr[n] != nnz"); return GC_EINVAL; }
    for (int64_t v = 0; v < n; ++v)
        if (row_ptr[v + 1] < row_ptr[v]) { gc_set_error("gc_graph_create: row_ptr not monotone at %lld", (long long)v); return GC_EINVAL; }
    gc_graph* g;
    int rc = new_graph(out, n, nnz, flags, &g);
    if (rc) return rc;
    int* raw = nullptr;
    if ((rc = alloc_scratch(g, &raw))) return rc;
    hipError_t e1 = hipMemcpy(g->rp, row_ptr, sizeof(long long) * (size_t)(n + 1), hipMemcpyHostToDevice);
    hipError_t e2 = nnz ? hipMemcpy(raw, col, sizeof(int) * (size_t)nnz, hipMemcpyHostToDevice) : hipSuccess;
    if (e1 != hipSuccess || e2 != hipSuccess) {
        gc_set_error("H2D copy failed");
        gc_dfree(raw);
        gc_free_all(g);
        delete g;
        return GC_EHIP;
    }
    return finish_create(g, out, raw, raw);
}

// The caller's device CSR is read in place (rp copied, col partitioned straight into the
// graph's own array): no device-to-device copy of the rows.  The caller's buffers must stay
// valid for the duration of the call only.
extern "C" int gc_graph_create_device(const int64_t* d_row_ptr, const int32_t* d_col, int64_t n, int64_t nnz,
                                      uint32_t flags, gc_graph** out) {
    if (!d_row_ptr || (nnz > 0 && !d_col)) { gc_set_error("gc_graph_create_device: null input"); return GC_EINVAL; }
    gc_graph* g;
    int rc = new_graph(out, n, nnz, flags, &g);
    if (rc) return rc;
    // the caller's CSR may still be being written on another stream (torch's); the library's
    // stream is non-blocking, so its first read is ordered after that stream's work (or after
    // all work on the device when the caller named no stream)
    if ((rc = gc_order_after_inputs(g->stream))) {
        gc_free_all(g);
        delete g;
        return rc;
    }
    if (hipMemcpyAsync(g->rp, d_row_ptr, sizeof(long long) * (size_t)(n + 1), hipMemcpyDeviceToDevice, g->stream) !=
        hipSuccess) {
        gc_set_error("D2D copy failed");
        gc_free_all(g);
        delete g;
        return GC_EHIP;
    }
    return finish_create(g, out, d_col, nullptr);
}

extern "C" int gc_graph_create_mesh(int64_t nx, int64_t ny, int64_t nz, gc_graph** out) {
    if (nx <= 0 || ny <= 0 || nz <= 0) { gc_set_error("mesh dims must be positive"); return GC_EINVAL; }
    const long long n = nx * ny * nz;
    const long long nnz = 2 * ((nx - 1) * ny * nz + nx * (ny - 1) * nz + nx * ny * (nz - 1));
    gc_graph* g;
    int rc = new_graph(out, n, nnz, GC_GRAPH_SYMMETRIC, &g);
    if (rc) return rc;
    int* raw = nullptr;
    if ((rc = alloc_scratch(g, &raw))) return rc;
    long long* cnt = nullptr;
    if (gc_raw_malloc((void**)&cnt, sizeof(long long) * (size_t)(n + 1)) != hipSuccess) {
        gc_dfree(raw); gc_free_all(g); delete g; gc_set_error("mesh alloc failed"); return GC_ENOMEM;
    }
    hipLaunchKernelGGL(k_mesh_deg, dim3(grid_for(n)), dim3(GC_BLOCK), 0, g->stream, nx, ny, nz, cnt);
    rc = exclusive_scan_ll(cnt, g->rp, n + 1, g->stream);
    hipFree(cnt);
    if (rc) { gc_dfree(raw); gc_free_all(g); delete g; return rc; }
    hipLaunchKernelGGL(k_mesh_fill, dim3(grid_for(n)), dim3(GC_BLOCK), 0, g->stream, nx, ny, nz, g->rp, raw);
    if (hipStreamSynchronize(g->stream) != hipSuccess) { gc_dfree(raw); gc_free_all(g); delete g; gc_set_error("mesh fill failed"); return GC_EHIP; }
    return finish_create(g, out, raw, raw);
}

// (the generator's key buffers are one-off: plain hipMalloc / hipFree, not the cache)
extern "C" int gc_graph_create_rmat(int32_t scale, int32_t edge_factor, double a, double b, double c, uint64_t seed,
                                    gc_graph** out) {
    if (scale < 1 || scale > 30 || edge_factor < 1 || a < 0 || b < 0 || c < 0 || a + b + c > 1.0) {
        gc_set_error("invalid R-MAT parameters");
        return GC_EINVAL;
    }
    const long long n = 1ll << scale;
    const long long m = (long long)edge_factor * n;
    const long long m2 = 2 * m;
    int dev = 0;
    hipGetDevice(&dev);
    hipStream_t s;
    GC_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    ull *k0 = nullptr, *k1 = nullptr;
    size_t* d_count = nullptr;
    void* tmp = nullptr;
    int* raw = nullptr;
    int rc = GC_OK;
    long long nuniq = 0, nnz = 0;
    gc_graph* g = nullptr;
    do {
        if (gc_raw_malloc((void**)&k0, sizeof(ull) * (size_t)m2) != hipSuccess ||
            gc_raw_malloc((void**)&k1, sizeof(ull) * (size_t)m2) != hipSuccess ||
            gc_raw_malloc((void**)&d_count, sizeof(size_t)) != hipSuccess) {
            gc_set_error("R-MAT key buffers (%lld keys) do not fit", m2);
            rc = GC_ENOMEM;
            break;
        }
        hipLaunchKernelGGL(k_rmat_edges, dim3(grid_for(m, 65536)), dim3(GC_BLOCK), 0, s, m, (int)scale, a, b, c,
                           (ull)seed, k0);
        size_t bytes = 0;
        rocprim::radix_sort_keys(nullptr, bytes, k0, k1, (size_t)m2, 0, 2 * scale, s);
        size_t bytes_u = 0;
        rocprim::unique(nullptr, bytes_u, k1, k0, d_count, (size_t)m2, rocprim::equal_to<ull>(), s);
        bytes = std::max(bytes, bytes_u);
        if (gc_raw_malloc(&tmp, bytes ? bytes : 1) != hipSuccess) { gc_set_error("sort temp alloc failed"); rc = GC_ENOMEM; break; }
        if (rocprim::radix_sort_keys(tmp, bytes, k0, k1, (size_t)m2, 0, 2 * scale, s) != hipSuccess ||
            rocprim::unique(tmp, bytes, k1, k0, d_count, (size_t)m2, rocprim::equal_to<ull>(), s) != hipSuccess) {
            gc_set_error("R-MAT sort/unique failed");
            rc = GC_EHIP;
            break;
        }
        size_t hcount = 0;
        hipMemcpyAsync(&hcount, d_count, sizeof(size_t), hipMemcpyDeviceToHost, s);
        if (hipStreamSynchronize(s) != hipSuccess) { gc_set_error("R-MAT generation failed"); rc = GC_EHIP; break; }
        nuniq = (long long)hcount;
        // last unique key may be the self-loop sentinel
        ull last = 0;
        if (nuniq > 0) hipMemcpy(&last, k0 + nuniq - 1, sizeof(ull), hipMemcpyDeviceToHost);
        const ull sentinel = (2 * scale == 64) ? ~0ull : ((1ull << (2 * scale)) - 1ull);
        nnz = (nuniq > 0 && last == sentinel) ? nuniq - 1 : nuniq;
        hipFree(k1);
        k1 = nullptr;
        hipFree(tmp);
        tmp = nullptr;
        hipSetDevice(dev);
        if ((rc = new_graph(out, n, nnz, GC_GRAPH_SYMMETRIC, &g))) break;
        if (gc_raw_malloc((void**)&raw, sizeof(int) * (size_t)std::max<long long>(nnz, 1)) != hipSuccess) {
            gc_set_error("R-MAT rows (%lld entries) do not fit", nnz);
            rc = GC_ENOMEM;
            break;
        }
        hipLaunchKernelGGL(k_keys_to_csr, dim3(grid_for(nnz, 65536)), dim3(GC_BLOCK), 0, s, k0, nnz, (int)scale, raw);
        hipLaunchKernelGGL(k_row_bounds, dim3(grid_for(n + 1, 65536)), dim3(GC_BLOCK), 0, s, k0, nnz, (int)scale, n,
                           g->rp);
        if (hipStreamSynchronize(s) != hipSuccess) { gc_set_error("R-MAT CSR build failed"); rc = GC_EHIP; break; }
    } while (0);
    if (k0) hipFree(k0);
    if (k1) hipFree(k1);
    if (tmp) hipFree(tmp);
    if (d_count) hipFree(d_count);
    hipStreamDestroy(s);
    if (rc) {
        if (raw) hipFree(raw);
        if (g) { gc_free_all(g); delete g; }
        return rc;
    }
    rc = finish_create(g, out, raw, nullptr);
    hipFree(raw);
    return rc;
}

// A graph with live shards (gc_shard_create borrows its rows and hub lists) is freed by the
// last gc_shard_destroy instead: freeing it here would leave the shards reading memory the
// caching allocator may already have handed to another graph.
extern "C" void gc_graph_destroy(gc_graph* g) {
    if (!g) return;
    if (g->shard_refs > 0) {
        g->destroy_pending = true;
        return;
    }
    gc_free_all(g);
    delete g;
}

extern "C" int gc_graph_info(const gc_graph* g, int64_t* n, int64_t* nnz, int64_t* max_degree, uint32_t* flags) {
    if (!g) { gc_set_error("null graph"); return GC_EINVAL; }
    if (n) *n = g->n;
    if (nnz) *nnz = g->nnz;
    if (max_degree) *max_degree = g->maxdeg;
    if (flags) *flags = g->flags;
    return GC_OK;
}

extern "C" int gc_graph_device(const gc_graph* g, int32_t* device) {
    if (!g || !device) { gc_set_error("null graph or output"); return GC_EINVAL; }
    *device = g->device;
    return GC_OK;
}

extern "C" int gc_graph_export(const gc_graph* g, int64_t* row_ptr, int32_t* col) {
    if (!g) { gc_set_error("null graph"); return GC_EINVAL; }
    GC_HIP(hipSetDevice(g->device));
    if (row_ptr) GC_READ(g->stream, (long long*)row_ptr, (const long long*)g->rp, (size_t)(g->n + 1));
    if (col && g->nnz) GC_READ(g->stream, (int*)col, (const int*)g->col, (size_t)g->nnz);
    return GC_OK;
}

extern "C" int gc_graph_export_device(const gc_graph* g, int64_t* d_row_ptr, int32_t* d_col) {
    if (!g) { gc_set_error("null graph"); return GC_EINVAL; }
    GC_HIP(hipSetDevice(g->device));
    if (d_row_ptr)
        GC_HIP(hipMemcpyAsync(d_row_ptr, g->rp, sizeof(long long) * (size_t)(g->n + 1), hipMemcpyDeviceToDevice, g->stream));
    if (d_col && g->nnz)
        GC_HIP(hipMemcpyAsync(d_col, g->col, sizeof(int) * (size_t)g->nnz, hipMemcpyDeviceToDevice, g->stream));
    GC_HIP(hipStreamSynchronize(g->stream));
    return GC_OK;
}

extern "C" int gc_graph_lower_counts(const gc_graph* g, int32_t* nlow_out) {
    if (!g || !nlow_out) { gc_set_error("null argument"); return GC_EINVAL; }
    GC_HIP(hipSetDevice(g->device));
    if (g->n) GC_READ(g->stream, (int*)nlow_out, (const int*)g->nlow, (size_t)g->n);
    return GC_OK;
}
