// gc_engine.h -- the gc_graph handle (internal; the ABI only sees an opaque pointer).
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <string>
#include <vector>

#include "gcolor.h"
#include "gc_launch.h"

struct gc_graph {
    int device = 0;
    long long n = 0, nnz = 0, maxdeg = 0;
    uint32_t flags = 0;
    // graph (HBM-resident)
    long long* rp = nullptr;
    int* col = nullptr;
    int* deg = nullptr;
    int* nlow = nullptr;       // lower-rank neighbours first in each row (see gc_graph.hip)
    long long* trp = nullptr;  // in-neighbour CSR; == rp/col when symmetric
    int* tcol = nullptr;
    // run state
    int* color = nullptr;
    int* cround = nullptr;
    int* cand = nullptr;
    unsigned char* c8 = nullptr;
    unsigned* c4 = nullptr;
    unsigned char* k8 = nullptr;
    unsigned* inF = nullptr;
    unsigned char* mark = nullptr;  // big-round push marks (zero between rounds)
    int* F[2] = {nullptr, nullptr};
    int* heavy = nullptr;
    int* wide = nullptr;
    int* undL[3] = {nullptr, nullptr, nullptr};
    int* undH[3] = {nullptr, nullptr, nullptr};
    int* seeds[2] = {nullptr, nullptr};
    int* bigw = nullptr;
    int* ulist = nullptr;
    int* parent = nullptr;
    ull* best = nullptr;
    int* vcolors = nullptr;
    int* lcur = nullptr;       // JP resume points (gc_jp_sweep)
    ull* bstat = nullptr;      // stats slots (gc_stat_add)
    ull* accs = nullptr;       // winner-count slots (k_commit -> k_close)
    // hubs (gc_hubs.hip), built on the first variant-A colouring that wants them
    int hub_t = -1;            // threshold they were built for (-1: none)
    int hub_w = 0;             // bitmap words per hub
    long long nhub = 0;
    int* hid = nullptr;
    int* hub_v = nullptr;
    long long* hin_rp = nullptr;
    int* hin_col = nullptr;
    unsigned* hbits = nullptr;
    unsigned* hkill = nullptr;
    long long* hlow_rp = nullptr;
    int* hlow_col = nullptr;
    int* hcur = nullptr;
    int* hpc = nullptr;
    int* hpend[2] = {nullptr, nullptr};
    int* hrow = nullptr;
    int* hlen = nullptr;
    int* hlow2[2] = {nullptr, nullptr};
    long long* hch_rp = nullptr;  // hub x: first static GC_HCH-entry chunk of its hlow row
    int* hch_own = nullptr;       // static chunk -> hub
    int* hkcnt = nullptr;         // hub x: kept-row entries written by the long-row first pass this round
    long long nhch = 0;           // static chunks
    unsigned* hk = nullptr;       // hub-indexed mirror of (candidate, JP state) (gc_hk; GC_HK_COLOURED)
    int* hcore = nullptr;         // hub core (gc_core.hip): hub -> core index, core index -> hub,
    int* core_hub = nullptr;      //   the core's bitsets and the build's per-workgroup counts
    unsigned* core_bits = nullptr;
    ull* core_wcnt = nullptr;
    int core_cap = 0;             //   the capacity they were allocated for
    unsigned* fsum = nullptr;  // per-workgroup counts of the frontier re-sort
    RoundRec* rec = nullptr;   // device round records
    long long rcap = 0;
    DevCtl* ctl = nullptr;
    DevCtl* hctl = nullptr;    // pinned host mirror
    DevCtl* hsnap = nullptr;   // pinned per-batch snapshots (2, pipelined)
    DevCtl* hsnap_dev = nullptr;  // the same, as the device addresses k_close writes them through
    hipEvent_t evsnap[2] = {nullptr, nullptr};
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::vector<hipEvent_t> evpool;
    bool has_run_state = false;
    bool borrowed = false;     // rp/col/deg/nlow belong to another handle (shard views)
    bool own_stream = true;    // false: the caller's stream (gc_shard_set_stream), not destroyed here
    int shard_refs = 0;        // live shards borrowing this graph's rows and hub lists (gc_shard_create)
    bool destroy_pending = false;  // gc_graph_destroy ran while shards lived: the last gc_shard_destroy frees it
    int part_prio = 0;         // rank the rows are partitioned for (gc_set_priority)
    int hub_prio = 0;          // row partition the hub lists were built under
    uint64_t hub_seed = 0;
    bool bpart = false;        // low parts also split by degree (variant B: equal-degree entries last, neq counts them)
    int* neq = nullptr;
    int* nhe = nullptr;        // per row: its entries of higher degree and earlier position (variant B's admission range end, gc_prep.hip)
    int* bpend = nullptr;      // variant B's pending entries (nnz ints, gc_color_variant_b allocates it)
    int* bwatch = nullptr;     // variant B: each undecided vertex's watched pending entry (n ints, likewise)
    int* hpl = nullptr;        // hubs-off heavy JP pending lists (gc_alloc_heavy_pending), nnz + n ints
    int* hplc = nullptr;
    uint64_t part_seed = 0;
    // edge-balanced tiling of the CSR (gc_prep.hip): whole-row tiles of <= GC_TW rows +
    // entries, rows longer than GC_TH split into GC_SEG-entry segments
    unsigned char* kb = nullptr;  // gc_deg_code(deg): the rank key's byte the partition gathers first
    int* tile_r0 = nullptr;       // [ntiles + 1] first row of each tile
    long long ntiles = 0;
    int* seg_row = nullptr;       // heavy segments: row, index within the row
    int* seg_j = nullptr;
    ull* seg_aux = nullptr;       // per segment: packed class counts of the last two-pass kernel
    unsigned* seg_cls = nullptr;  // per segment and thread: 16 x 2-bit classes
    long long* seg_base = nullptr;  // [ntiles + 1] exclusive scan of the tiles' segment counts; [ntiles] = total
    long long nseg_cap = 0;
    unsigned* hubmap = nullptr;   // bit per vertex: hid >= 0
    unsigned* hubpre = nullptr;   // hubs in the words before (id-order index of a hub = hubpre + rank in its word)
    int* hperm = nullptr;         // id-order index -> hub index (rank order)
    ull* hb_bits = nullptr;       // hub-transpose build only: bit per entry (col[e] is a hub)
    long long* hb_wpre = nullptr; //   and the exclusive prefix of the words' popcounts
    uint2* hb_mp = nullptr;       //   and hubmap / hubpre interleaved per word
    // by-product of the creation's rank partition (symmetric graphs): byte e = 1 iff col[e] is
    // a hub (deg > hubflag_t) -- the hub transpose's count pass then streams these bytes
    // instead of gathering a hub bit per entry; freed by that pass or by a re-partition
    unsigned char* hubflag = nullptr;
    int hubflag_t = -1;
};

// caching allocator (gc_alloc.hip): every device / pinned-host buffer of the library
hipError_t gc_dmalloc(void** p, size_t bytes);
hipError_t gc_hmalloc(void** p, size_t bytes);
hipError_t gc_dfree(void* p);
size_t gc_cache_idle_bytes(void);  // parked bytes (count as free memory)
hipError_t gc_raw_malloc(void** p, size_t bytes);  // uncached (one-off buffers); releases the cache on failure

// gc_prep.hip: tiling, rank partition, validation and hub-transpose passes
int gc_build_tiling(gc_graph* g);
// rank partition of rows (rp, src) into dst (!= src): per row [class 0 | class 1 | class 2]
// with class 0 = lower key, 1 = equal key and earlier position (both lower rank), 2 =
// higher rank; nlow = c0 + c1, neq = c1 (neq may be null).  prio 0: key = deg (coloring.py:64),
// 1: key = prio_hash(seed, v).  *bad (device) counts entries outside [0, n).
int gc_partition(gc_graph* g, const int* src, int* dst, int prio, uint64_t seed, ull* bad,
                 unsigned char* hubflag = nullptr, int hub_t = -1);
// the hub threshold of the colourings (GC_HUB_T, "off" or < 0: none; default GC_HUB_T)
int gc_hub_threshold();
// whether the rank partition can mark hub entries (gc_prep.hip: 3 bits per entry in seg_cls)
bool gc_partition_hubflags_supported();
// -> ctl->uncolored, ctl->conflicts; c8 (optional): the byte mirror of `colors` (the resident colouring)
int gc_validate_tiles(gc_graph* g, const int* colors, const unsigned char* c8, long long lo, long long hi);
// symmetric graphs: hub transpose (hin_rp / hin_col: the hubs listed in each row) and the
// lower-rank hubs of every hub row (hlow counts -> klow[x]); hubmap / hid / hub_v ready
int gc_hub_transpose_sym(gc_graph* g, long long H, long long* hin_rp, long long* klow, int T);
int gc_hub_transpose_fill(gc_graph* g, long long H);
void gc_hub_bits_free(gc_graph* g);

void gc_set_error(const char* fmt, ...);

#define GC_HIP(call)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (call);                                                               \
        if (e_ != hipSuccess) {                                                               \
            gc_set_error("%s failed at %s:%d: %s", #call, __FILE__, __LINE__, hipGetErrorString(e_)); \
            return GC_EHIP;                                                                   \
        }                                                                                     \
    } while (0)

// Host reads of device data produced on a stream (counts, offsets, exports): the copy is
// enqueued on THAT stream and waited for with its status checked.  A plain hipMemcpy does not
// wait for the library's non-blocking streams (round 4's k_hin_fill fault: hin_col was sized
// from a stale count), and a failure of an earlier kernel is reported here, at the read that
// depends on it, instead of at a later unrelated call.
template <typename T>
inline int gc_read_dev(hipStream_t s, T* host, const T* dev, size_t count = 1) {
    if (count == 0) return GC_OK;
    hipError_t e = hipMemcpyAsync(host, dev, sizeof(T) * count, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        gc_set_error("device-to-host read of %zu bytes: %s", sizeof(T) * count, hipGetErrorString(e));
        return GC_EHIP;
    }
    return GC_OK;
}
#define GC_READ(s, host, dev, count)                             \
    do {                                                         \
        const int rr_ = gc_read_dev((s), (host), (dev), (count)); \
        if (rr_) return rr_;                                     \
    } while (0)

// Order the library stream `s` after the caller's device inputs: an event on the stream set
// with gc_set_input_stream (this thread), else a device-wide synchronisation.
int gc_order_after_inputs(hipStream_t s);

int gc_alloc_graph_common(gc_graph* g, const int* src);  // deg, maxdeg, rank partition of src, transpose (gc_graph.hip)
int gc_build_in_csr(gc_graph* g, long long lo, long long hi);  // in-neighbour CSR of rows [lo, hi)
int gc_build_in_csr_sym(gc_graph* g, long long lo, long long hi);  // the same, symmetric graphs (no atomics)
int gc_filter_rows_sym(gc_graph* g, gc_graph* v, long long lo, long long hi);  // the same over g's tiling (gc_prep.hip)
int gc_alloc_run_state(gc_graph* g);     // gc_engine.hip
int gc_hubs_prepare(gc_graph* g, GDev& d);
int gc_core_prepare(gc_graph* g, GDev& d);  // gc_core.hip: the hub core's buffers (once per graph); d.core_cap
int gc_alloc_heavy_pending(gc_graph* g);  // gc_engine.hip: the hubs-off heavy JP's pending lists, on first use  // gc_hubs.hip: build (once) + reset; fills d's hub fields
void gc_hubs_free(gc_graph* g);
int gc_color_variant_b(gc_graph* g, const gc_options* opt, int32_t* colors_out, int32_t* cround_out,
                       gc_stats* st);  // gc_variant_b.hip
void gc_free_all(gc_graph* g);
int gc_set_priority(gc_graph* g, int prio, uint64_t seed);  // gc_priority.hip: rows partitioned for the rank
int gc_color_speculative(gc_graph* g, const gc_options* opt, int32_t* colors_out, int32_t* cround_out,
                         gc_stats* st);  // gc_priority.hip
GDev gc_view(const gc_graph* g);
GLists gc_lists(const gc_graph* g);
static inline int gc_grid_for_waves(long long items, int cap = 2048) {
    long long chunks = (items + GC_WAVE - 1) / GC_WAVE;
    long long blocks = (chunks + GC_WAVES_PER_BLOCK - 1) / GC_WAVES_PER_BLOCK;
    if (blocks < 1) blocks = 1;
    if (blocks > cap) blocks = cap;
    return (int)blocks;
}

// Per-class HIP-event timing of a colouring's launches (gc_options.kernel_timing): begin(cls)
// before a launch opens a run of that class (consecutive launches of one class share it),
// collect() adds the runs' times to gc_stats.k_ms.  Used by the one-GPU engine and variant B.
#include <stdio.h>
#include <stdlib.h>
struct KTimer {
    gc_graph* g;
    unsigned mask;  // kernel classes to time (bit GC_K_*)
    gc_stats* st;
    int run_cls = -1;  // class of the open run (-1: none)
    int cnt_cls = -1;  // class the launches since cnt_start are counted for (timed or not)
    long long cnt_start = 0;
    std::vector<std::pair<int, size_t>> recs;  // (class, event index of start)
    size_t used = 0;
    hipEvent_t ev() {
        if (used >= g->evpool.size()) {
            hipEvent_t e;
            hipEventCreate(&e);
            g->evpool.push_back(e);
        }
        return g->evpool[used++];
    }
    // GC_DEBUG_SYNC: synchronise after every launch and name the kernel class of a fault
    const bool dbg_sync = getenv("GC_DEBUG_SYNC") != nullptr;
    int last_cls = -1;
    long long nlaunch = 0;
    // the kernels launched (GC_LAUNCH) since the class was begun go to its k_launches
    void count() {
        if (cnt_cls >= 0 && st) st->k_launches[cnt_cls] += gc_tl_launches - cnt_start;
        cnt_cls = -1;
    }
    void begin(int cls) {
        last_cls = cls;
        ++nlaunch;
        if (cls != cnt_cls) {
            count();
            cnt_cls = cls;
            cnt_start = gc_tl_launches;
        }
        if (cls == run_cls) return;  // the open run goes on
        close();
        if (!((mask >> cls) & 1u)) return;
        run_cls = cls;
        recs.push_back({cls, used});
        hipEventRecord(ev(), g->stream);
    }
    void end() {
        if (!dbg_sync) return;
        const hipError_t e = hipStreamSynchronize(g->stream);
        if (e != hipSuccess) {
            fprintf(stderr, "[gc debug-sync] launch %lld (class %d) failed: %s\n", nlaunch, last_cls, hipGetErrorString(e));
            fflush(stderr);
            abort();
        }
    }
    void close() {
        if (run_cls < 0) return;
        hipEventRecord(ev(), g->stream);
        run_cls = -1;
    }
    void collect() {
        close();
        count();
        if (!mask || !st) return;
        for (auto& r : recs) {
            float ms = 0.f;
            hipEventElapsedTime(&ms, g->evpool[r.second], g->evpool[r.second + 1]);
            st->k_ms[r.first] += ms;
        }
    }
};

