/*
 * gcolor.h -- C-ABI of the MI355X-native graph-colouring engine (libgcolor.so).
 *
 * This is the drop-in boundary for the reference's hot path.  The reference exposes no
 * FFI; its in-process surface is two Python functions that this ABI replaces:
 *
 *   graph_coloring(graph_rdd, numOfColors, sc) -> (bool, rdd)   /root/reference/coloring.py:73
 *        (variant B: /root/reference/coloring_optimized.py:70)     -> gc_color()
 *   validate_graph_coloring(graph_rdd) -> bool                     /root/reference/coloring.py:149
 *                                                                   -> gc_validate()
 *   the Spark data model (Node objects in an RDD, node.py:1-18,     -> gc_graph (device CSR)
 *        graph.py:15-28, coloring.py:201-209)
 *   Graph(node_count, max_degree) generator, graph.py:30-43        -> gc_gen_uniform()
 *
 * Conventions: every function is extern "C", never throws, returns an int status
 * (GC_OK == 0) unless it returns void/const char*; host arrays are caller-owned;
 * device memory is owned by the gc_graph handle.  One handle per calling thread.
 * Vertices are FILE POSITIONS 0..n-1 (the caller maps JSON ids); adjacency lists are
 * kept exactly as listed (duplicates, self-loops and asymmetric lists are legal and
 * keep the reference's directed semantics).
 */
#ifndef GCOLOR_H
#define GCOLOR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------------------ */
#define GC_OK 0
#define GC_FAILED 1    /* bounded attempt: a proposer's mex >= num_colors (coloring.py:104-108) */
#define GC_STALLED 2   /* zero proposers, uncoloured vertices left, E1 off (coloring.py:93-95)  */
#define GC_EINVAL (-1)
#define GC_EHIP (-2)
#define GC_ENOMEM (-3)
#define GC_ERCCL (-4)
#define GC_EROUNDS (-5)
#define GC_EUNSUPPORTED (-6) /* JSON the native reader leaves to Python's json + graph.py rules  */
#define GC_EKEY (-7)         /* neighbour id that is no node id: KeyError (gc_last_error() = id)  */
#define GC_EIO (-8)

/* ---- graph -------------------------------------------------------------------------- */
typedef struct gc_graph gc_graph;

#define GC_GRAPH_SYMMETRIC 1u /* caller asserts (v,u) listed <=> (u,v) listed: no transpose kept */

/* Copy a host CSR (row_ptr int64[n+1], col int32[nnz] of positions) to the device.
   Replaces: sc.parallelize(graph.nodes)...persist(), coloring.py:201-209.           */
int gc_graph_create(const int64_t* row_ptr, const int32_t* col, int64_t n, int64_t nnz,
                    uint32_t flags, gc_graph** out);
/* Same, from device pointers already resident in HBM: rp is copied, the rows are read in
   place and written rank-partitioned into the graph's own array (no copy of col).  The
   caller's buffers need to stay valid only for the duration of the call.  Ordering: the
   library works on its own non-blocking stream, so its first read is ordered after the
   stream named with gc_set_input_stream (an event wait), or -- when none is named -- after
   all work on the device (hipDeviceSynchronize): buffers still being written by kernels on
   another stream (e.g. torch's) are complete before their first read.                  */
int gc_graph_create_device(const int64_t* d_row_ptr, const int32_t* d_col, int64_t n, int64_t nnz,
                           uint32_t flags, gc_graph** out);
/* Device-side synthetic generators (no host round trip):
   R-MAT (a,b,c; d = 1-a-b-c), 2^scale vertices, edge_factor*2^scale generated edges,
   self-loops dropped, symmetrised, de-duplicated, rows sorted, no vertex permutation. */
int gc_graph_create_rmat(int32_t scale, int32_t edge_factor, double a, double b, double c,
                         uint64_t seed, gc_graph** out);
/* 3-D 7-point mesh, id = x + nx*(y + ny*z), neighbours in order -x,+x,-y,+y,-z,+z.   */
int gc_graph_create_mesh(int64_t nx, int64_t ny, int64_t nz, gc_graph** out);
void gc_graph_destroy(gc_graph* g);
int gc_graph_info(const gc_graph* g, int64_t* n, int64_t* nnz, int64_t* max_degree, uint32_t* flags);
/* The HIP device the graph lives on (the current device when it was created).        */
int gc_graph_device(const gc_graph* g, int32_t* device);
/* Copy the device CSR back (row_ptr int64[n+1], col int32[nnz]); either may be NULL.
   Rows come back in the engine's order: each row lists its lower-rank neighbours
   (rank = (deg, pos), coloring.py:64) first -- the same multiset as the input row.   */
int gc_graph_export(const gc_graph* g, int64_t* row_ptr, int32_t* col);
/* The same into caller-owned DEVICE buffers (device-to-device; either may be NULL).    */
int gc_graph_export_device(const gc_graph* g, int64_t* d_row_ptr, int32_t* d_col);
/* nlow_out (host int32[n]): how many entries at the head of each exported row rank
   below the row's vertex.                                                            */
int gc_graph_lower_counts(const gc_graph* g, int32_t* nlow_out);

/* ---- colouring ---------------------------------------------------------------------- */
#define GC_VARIANT_A 0 /* coloring.py (default)           */
#define GC_VARIANT_B 1 /* coloring_optimized.py           */

#define GC_PRIORITY_REF 0    /* rank (deg, pos): the reference's tie-break, coloring.py:64     */
#define GC_PRIORITY_SEEDED 1 /* rank (prio_hash(seed, v), pos): seeded priorities (north_star) */

typedef struct gc_options {
    int32_t variant;       /* GC_VARIANT_A / GC_VARIANT_B                                  */
    int32_t e1;            /* 1: re-seed on a zero-proposer round (extension E1)           */
    int64_t num_colors;    /* k of graph_coloring(graph, k); < 0 = unbounded               */
    int32_t kernel_timing; /* bit GC_K_x set: time that class's launches with HIP events
                              (gc_stats.k_ms); 0xFF = every class, 0 = none             */
    int32_t priority;      /* GC_PRIORITY_REF / GC_PRIORITY_SEEDED (variant A only): the rank
                              that orders each colour's conflict resolution             */
    uint64_t seed;         /* seed of GC_PRIORITY_SEEDED                                    */
    int32_t speculative;   /* 1: speculative first-fit rounds -- every uncoloured vertex
                              proposes, one-shot resolution under the rank (variant A
                              only; not the reference's semantics: valid colourings,
                              colour count reported against the reference)              */
    int32_t reserved;
} gc_options;

/* kernel classes reported in gc_stats.k_* */
#define GC_K_INIT 0
#define GC_K_PROPOSE 1
#define GC_K_RESOLVE 2
#define GC_K_SWEEP 3
#define GC_K_COMMIT 4
#define GC_K_RESEED 5
#define GC_K_VALIDATE 6
#define GC_K_OTHER 7
#define GC_NKERNELS 8

typedef struct gc_stats {
    /* outputs */
    int64_t rounds;        /* rounds run; the per-round arrays hold the first min(rounds,
                              round_cap) of them (a caller short of room asks again)     */
    int64_t fail_round;    /* bounded attempt: round that failed, else -1                 */
    int64_t fail_count;    /* #proposers with mex >= k in that round                      */
    int64_t reseeds;       /* E1 seeds planted                                            */
    int64_t max_color;     /* max colour of the final state (-1: none)                    */
    int64_t jp_sweeps;     /* Jones-Plassmann sweeps beyond the first, summed over rounds */
    double device_ms;      /* HIP-event time of the whole colouring (resident CSR in)     */
    int64_t k_launches[GC_NKERNELS];
    double k_ms[GC_NKERNELS];    /* valid when kernel_timing = 1                           */
    double k_bytes[GC_NKERNELS]; /* algorithmic bytes per kernel class     */
    /* optional caller buffers (may be NULL), capacity round_cap */
    int64_t round_cap;
    int64_t* round_U;      /* uncoloured at round start (coloring.py:89 transcript)        */
    int64_t* round_F;      /* proposers                                                   */
    int64_t* round_maxmex; /* max candidate colour proposed (-1 if none)                  */
    int64_t* round_accepted;
    int64_t* round_seeds;  /* E1 seeds planted in the round                               */
    /* outputs (continued) */
    int64_t async_aborts;  /* asynchronous JP launches that handed their rest to host
                              sweeps at their time budget (diagnostic; 0 expected)        */
    int64_t hubs;          /* vertices with pushed hub state (forbidden-colour bitmaps) in
                              this colouring; 0 when none is above the hub threshold or the
                              hub index did not fit (then gc_color printed a warning)      */
    int64_t core_rounds;   /* rounds whose hub JP the hub core decided in one workgroup
                              (k_hub_core, csrc/gc_core.hip); the rest went through the
                              asynchronous JP (diagnostic)                                 */
} gc_stats;

/* Colour the graph.  colors_out (host int32[n], may be NULL): final state, -1 =
   uncoloured; on GC_FAILED it is the state at the START of the failing round, exactly
   what graph_coloring returns with False.  colored_round_out (host int32[n], may be
   NULL): round at whose start each vertex was coloured (0 = init/seed, -1 = never). */
int gc_color(gc_graph* g, const gc_options* opt, int32_t* colors_out, int32_t* colored_round_out,
             gc_stats* stats);

/* The same colouring continued from round `round0` of a run in progress (variant A, reference
   rank): colors_dev (DEVICE int32[n], -1 = uncoloured) are the colours so far, front_dev
   (DEVICE int32[nfront]) the uncoloured vertices with a coloured listed neighbour (each
   once, any order), cround_dev (DEVICE int32[n] or NULL) the round each was coloured in.
   Replaces coloring.py:73-132 from that round on; stats hold the rounds from round0 (their
   records, the failing round as an absolute index).  The multi-GPU hybrid hands the
   replicated state of its sharded rounds to the one-GPU engine with it.  Ordering: as
   gc_graph_create_device, the device buffers are read after all work on the device.     */
int gc_color_resume(gc_graph* g, const gc_options* opt, const int32_t* colors_dev, const int32_t* cround_dev,
                    const int32_t* front_dev, int64_t nfront, int64_t round0, int32_t* colors_out,
                    int32_t* colored_round_out, gc_stats* stats);

/* validate_graph_coloring counts: #uncoloured and the directed count of listed pairs
   (v, u in N(v)) with colour[u] == colour[v] (self-loops and duplicates count, as in
   coloring.py:157-158).  colors == NULL validates the device result of the last
   gc_color on this handle without a host round trip.
   On a graph created with GC_GRAPH_SYMMETRIC the count is 2 x the conflicts of the rows'
   lower-rank entries + the self-loop entries (half the gathers; GC_VALIDATE_HALF=0 counts
   every entry): exact when the rows ARE symmetric, which the flag asserts -- the library does
   not check it.  Create an asymmetric graph without the flag (then every entry is counted).  */
int gc_validate(gc_graph* g, const int32_t* colors, int64_t* uncolored, int64_t* conflicts);

/* The same counts over the rows of vertices [lo, hi) only: every uncoloured vertex of the
   range and every conflicting listed pair (v, u) with v in the range.  Disjoint ranges that
   cover [0, n) add up to gc_validate's counts, so ranks that each hold the colouring split
   validate_graph_coloring (coloring.py:149-162) by vertex range and sum the two counts (the
   multi-GPU bench step: one all-reduce).  On a graph created GC_GRAPH_SYMMETRIC (and
   GC_VALIDATE_HALF on, the default) a conflicting pair is counted twice from the row of its
   HIGHER-rank end -- the row whose lower-rank part lists the other end -- as gc_validate does,
   so the count of one range is not the conflicts of its own rows: only the sum over disjoint
   ranges covering [0, n) is meaningful.  GC_VALIDATE_HALF=0 counts every listed entry of the
   range's rows (then a range's count is its rows' own).                                      */
int gc_validate_range(gc_graph* g, const int32_t* colors, int64_t lo, int64_t hi, int64_t* uncolored,
                      int64_t* conflicts);

/* ---- multi-GPU shards ------------------------------------------------ */
/* One rank's share of a colouring on the graph g (every rank holds the whole CSR): the
   rank owns vertices [lo, hi) and runs the round on its own frontier.  A round is cut at
   its grid-wide seams -- propose and the Jones-Plassmann sweeps -- where the rank
   publishes what changed on its own vertices: int64 deltas (vertex << 32 | value) in a
   caller-owned DEVICE buffer (capacity >= hi - lo), or its slice of the proposal bytes,
   and takes everyone's back (gc_shard_apply / gc_shard_put_slices).  After the last
   sweep seam every rank colours all winners itself (gc_shard_finish).  The caller moves
   the data between ranks (RCCL all-gather in gcolor_amd/shard.py).  The colouring is
   bit-identical to gc_color on one GPU.
   Replaces: the Spark shuffle/broadcast of each round (coloring.py:82-83, 110-127).  */
typedef struct gc_shard gc_shard;
#define GC_KIND_CAND 0   /* (v, candidate): propose seam                                */
#define GC_KIND_STATE 1  /* (v, 1 = IN | 2 = OUT): JP sweep seam                        */
#define GC_KIND_COLOUR 2 /* (v, colour): colours set elsewhere                          */
int gc_shard_create(gc_graph* g, int64_t lo, int64_t hi, gc_shard** out);
void gc_shard_destroy(gc_shard* s);
/* init + seed (coloring.py:12-35) on the replicated state; *U_out global uncoloured,
   *F_out this rank's frontier                                                         */
int gc_shard_begin(gc_shard* s, int64_t num_colors, int32_t track_rounds, int64_t* U_out, int64_t* F_out);
/* stats[4]: deltas written, frontier size, max candidate (-1 none), #candidates >= k    */
int gc_shard_propose(gc_shard* s, int64_t round, int64_t* delta, int64_t cap, int64_t* stats);
int gc_shard_apply(gc_shard* s, int32_t kind, const int64_t* recv, int64_t count, int64_t round);  /* enqueued */
/* Fused propose seam (the first JP sweep enqueued behind it, no host wait between): recv is
   every rank's send buffer of hdr_stride words; nothing is applied and the shard halts
   (GC_H_SEAM = 7: its kernels do nothing) when some rank's header shows a halted finish or
   more deltas than fit inline -- the caller then clears it (gc_shard_clear_halt) and takes
   the unfused path.                                                                       */
int gc_shard_apply_checked(gc_shard* s, int32_t kind, const int64_t* recv, int64_t count, int64_t round,
                           int64_t hdr_stride);
int gc_shard_clear_halt(gc_shard* s, int32_t code);  /* halt := run if it is `code` (enqueued) */
/* the same phases, only enqueued (no wait, no stats): their counts travel in the seam's
   header, written on the device by gc_shard_pack                                        */
int gc_shard_propose_async(gc_shard* s, int64_t round, int64_t* delta, int64_t cap);
int gc_shard_sweep_async(gc_shard* s, int32_t i, int32_t count, int64_t* delta, int64_t cap);
/* a seam's send buffer (device, 5 + cap int64): 5 header words -- propose: frontier, max
   candidate, #candidates >= k, #deltas, winners of the last finished round (or -halt code
   when that finish halted: gc_shard_resume_hubs); sweep: undecided in list slot `slot`
   (+ hubs waiting for gc_shard_start_hubs), #deltas, undecided light vertices, #deltas,
   0 -- each encoded (0xFFFFFFFF << 32 | value) so appliers skip it as padding, then
   up to cap deltas padded with -1 (delta == NULL: the header only)                      */
int gc_shard_pack(gc_shard* s, int32_t kind, int32_t slot, const int64_t* delta, int64_t* send, int64_t cap);
/* sweeps i .. i+count-1 (i = 0: first sweep over the frontier, then over the undecided);
   delta may be NULL (slice seam).  stats[2]: deltas written, still undecided here      */
int gc_shard_sweep(gc_shard* s, int32_t i, int32_t count, int64_t* delta, int64_t cap, int64_t* stats);
/* Replicated hubs (default; GC_SHARD_HUBS=0 at gc_shard_create turns them off): every rank
   holds and runs the hub state of every high-degree vertex, so hubs never travel.
   *nhub = the number of replicated hubs (0: none, hubs resolve through the seams).  Once a
   sweep seam reports no undecided light vertex on any rank (header word 2 == 0 on every
   rank) while vertices are still undecided (word 0), gc_shard_start_hubs runs the hubs'
   sweeps i, i+1, ... to their end with no exchange (from_slices = 1: a slice seam moved
   light states this round); *sweeps_out = sweeps run.                                  */
int gc_shard_hub_count(gc_shard* s, int64_t* nhub);
int gc_shard_start_hubs(gc_shard* s, int32_t i, int32_t from_slices, int64_t* sweeps_out);
/* The same, only enqueued: `grid` full-grid hub sweeps from i, then the one-workgroup tail
   (no host wait); gc_shard_finish_async(check = 1) verifies on the device that the hub JP
   converged, else the round halts and the next propose seam's header word 4 reads
   -GC_H_SWEEPS (5) on every rank: gc_shard_resume_hubs runs the rest, then the caller
   enqueues the finish again and repeats the propose seam.                              */
int gc_shard_start_hubs_async(gc_shard* s, int32_t i, int32_t from_slices, int32_t grid);
int gc_shard_resume_hubs(gc_shard* s, int64_t* sweeps_out);
/* slice seam: the rank's slice [lo, hi) of the proposal bytes (cand6 << 2 | JP state)
   into dst (device, hi - lo bytes); put_slices copies the other ranks' slices back    */
int gc_shard_get_slice(gc_shard* s, uint8_t* dst);
int gc_shard_put_slices(gc_shard* s, const uint8_t* src, int64_t stride, const int64_t* starts,
                        const int64_t* lens, int32_t parts);
/* end of round: colour ALL ranks' winners -- from the IN state deltas applied this round
   (from_deltas = 1: every sweep seam moved deltas) or read off the replicated proposal
   bytes -- push them into the rank's in-neighbours; *acc_out = winners (global), *F_out =
   new frontier                                                                         */
int gc_shard_finish(gc_shard* s, int64_t round, int32_t from_deltas, int64_t* acc_out, int64_t* F_out);
/* the same, only enqueued (no wait): the winners' count arrives in the next propose seam's
   header (word 4); check = 1 after gc_shard_start_hubs_async                            */
int gc_shard_finish_async(gc_shard* s, int64_t round, int32_t from_deltas, int32_t check);
/* run the shard's kernels on the caller's stream (a hipStream_t, e.g. torch's current one,
   where the collectives run): apply / get_slice / put_slices then only enqueue          */
int gc_shard_set_stream(gc_shard* s, void* stream);
/* E1 re-seed on the replicated state (same seeds on every rank)                        */
int gc_shard_reseed(gc_shard* s, int64_t round, int64_t* nseeds, int64_t* F_out);
int gc_shard_colors(gc_shard* s, int32_t* colors_out, int32_t* colored_round_out);
/* The replicated colours / rounds into DEVICE buffers and the rank's own frontier of the
   current round (DEVICE int32, capacity hi - lo; *nfront = its length): the state
   gc_color_resume continues from.                                                      */
int gc_shard_export(gc_shard* s, int32_t* colors_dev, int32_t* colored_round_dev, int32_t* front_dev,
                    int64_t* nfront);

/* ---- host-side generator ------------------------------------------------------------ */
/* The graph.py:30-43 process (per node: target = U{0..D}; draw random partners, keep
   those that are not self, not yet adjacent and below D) with a splitmix64 stream
   instead of Python's MT19937.  row_ptr int64[n+1]; col capacity col_cap (n*D is
   always enough); *nnz_out receives the entry count.                                 */
int gc_gen_uniform(int64_t n, int32_t max_degree, uint64_t seed, int64_t* row_ptr, int32_t* col,
                   int64_t col_cap, int64_t* nnz_out);

/* ---- graph files ------------------------------------------- */
/* A host CSR owned by the library (free with gc_csr_free).  ids: the JSON node ids in
   file order (NULL for a GCSR file written without ids: ids = positions).            */
typedef struct gc_csr {
    int64_t n, nnz;
    int64_t* row_ptr; /* int64[n+1] */
    int32_t* col;     /* int32[nnz], file positions */
    int64_t* ids;     /* int64[n] or NULL */
    uint32_t flags;   /* GC_GRAPH_SYMMETRIC when the writer asserted it */
} gc_csr;
/* The reference's JSON graph -> CSR over file positions.
   Replaces: Graph.deserialize_graph, graph.py:15-28 (json.load + id -> Node linking).
   Exact on what it accepts (int64 ids, integer neighbour lists, strict JSON); a repeated
   id resolves to its LAST node (graph.py:23); the first unknown neighbour id in file
   order returns GC_EKEY with the id as the message (graph.py:25 KeyError).  Anything
   else returns GC_EUNSUPPORTED and the caller applies Python's own rules.            */
int gc_json_read_graph(const char* path, gc_csr** out);
/* json.dump(result, f, indent=4) of [{"id", "color"}] (coloring.py:238-241) and of
   [{"id", "neighbors", "color"}] (graph.py:10-12, node.py:8-13), byte-identical to
   Python's encoder.  ids may be NULL (ids = positions); colors NULL writes -1.        */
int gc_json_write_coloring(const char* path, const int64_t* ids, const int32_t* colors, int64_t n);
int gc_json_write_graph(const char* path, const int64_t* ids, const int64_t* row_ptr, const int32_t* col,
                        int64_t n, const int32_t* colors);
/* Binary CSR (.gcsr) for graphs beyond JSON scale; layout in csrc/gc_io_host.cpp.     */
int gc_csr_write(const char* path, const int64_t* row_ptr, const int32_t* col, const int64_t* ids, int64_t n,
                 int64_t nnz, uint32_t flags);
int gc_csr_read(const char* path, gc_csr** out);
void gc_csr_free(gc_csr* c);

/* ---- misc ----------------------------------------------------------------------------- */
const char* gc_last_error(void);
/* Return every device / pinned block the library's allocator has parked for reuse (graph
   handles that are created and destroyed repeatedly get their buffers from that cache).  */
int gc_release_cache(void);
/* The stream (a hipStream_t, e.g. torch's current one) on which this thread's device inputs
   to gc_graph_create_device / gc_color_resume are produced: those calls then order their
   first read after it with an event instead of synchronising the whole device (which waits
   for other threads' work too and is invalid during a stream capture).  enable = 0 restores
   the device-wide synchronisation.  Per thread.                                         */
int gc_set_input_stream(void* stream, int32_t enable);
int gc_device_count(int32_t* count);
int gc_set_device(int32_t device);

#ifdef __cplusplus
}
#endif
#endif /* GCOLOR_H */
