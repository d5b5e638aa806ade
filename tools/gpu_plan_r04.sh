#!/bin/bash
# Round 4's GPU sessions, one gpurun call each (<= 1200 s):
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash tools/gpu_plan_r04.sh a
#   a: the stage-overflow corner first (round 3's k_commit fault, fixed by GC_COUNT_MASK and
#      now bounded by the list capacity in every build), then every GPU test, smoke, the
#      bench line with its rocprofv3 trace + FETCH/WRITE PMC passes (profiles/pmc of THIS
#      build), and the hubs-off asynchronous JP that faulted in round 3, last
set -uo pipefail
cd "$(dirname "$0")/.."
case ${1:-} in
  a) exec_steps=(staged:overflow_tree staged:under_ticket_close tests smoke profile:rmat24 staged:async_jp_without_hubs) ;;
  # b: every staged path's parity tests, each a soft step (a plain test failure is recorded and
  #    the session goes on; a GPU error still ends it), then the per-round cost by frontier size
  b) exec_steps=("?staged:resume~or~hybrid" "?staged:b_async" "?staged:async_resolve" "?staged:big_close"
                 "?staged:test_graphs_" "?staged:small_grid" "?staged:validate_c8" ubench:launch_gap rounds:rmat24) ;;
  # c: interleaved in-process A/Bs of the environment knobs, then the compile-time variants
  c) exec_steps=(ab:rmat24:6:base,ares=GC_ASYNC_RESOLVE:1,bclose=GC_BIG_CLOSE:1,graphs=GC_GRAPHS:1,small=GC_GRID_SMALL:256,bpc4=GC_ASYNC_BPC:4
                 ab:uniform10M:8:base,async2=GC_ASYNC:2,graphs=GC_GRAPHS:1,small=GC_GRID_SMALL:256
                 ab:mesh512:4:base,graphs=GC_GRAPHS:1,async2=GC_ASYNC:2
                 env:AB_VARIANT=B ab:rmat24:3:base,basync=GC_B_ASYNC:1 env:AB_VARIANT=
                 abl:rmat24:4:2:base=-,marks4=variants/marks4/libgcolor.so,claim4=variants/claim4/libgcolor.so,all4=variants/all4/libgcolor.so,hinhoist=variants/hinhoist/libgcolor.so,closeint=variants/close_interleaved/libgcolor.so,closecall=variants/close_call/libgcolor.so,tile8=variants/tile8/libgcolor.so) ;;
  # d: variant B's profile (PMC of this build), the tile size on the other workloads, the
  #    validation from the byte mirror, and the hybrid's switch point at P = 1
  d) exec_steps=(file:tests/test_gpu_hubs.py file:tests/test_gpu_parity.py env:GC_PREP_TIMING=1 step:rmat26 env:GC_PREP_TIMING=
                 "profile:rmat24:--variant,B"
                 abl:rmat26:3:1:base=-,tile8=variants/tile8/libgcolor.so,base2=-
                 abl:uniform10M:6:1:base=-,tile8=variants/tile8/libgcolor.so
                 abl:mesh512:3:1:base=-,tile8=variants/tile8/libgcolor.so
                 ab:rmat26:3:base,c8=GC_VALIDATE_C8:1 ab:rmat24:5:base,c8=GC_VALIDATE_C8:1
                 "bench:rmat24:--sharded,--multi,hybrid,--switch-below,1000000000,--steps,3,--warmup,1"
                 "bench:rmat24:--sharded,--multi,hybrid,--switch-below,262144,--steps,3,--warmup,1"
                 "bench:rmat24:--sharded,--multi,hybrid,--switch-below,16384,--steps,3,--warmup,1") ;;
  # e: after d's fault (the host read hin_rp[n] before the stream finished: fixed by a stream
  #    synchronisation in gc_hub_transpose_sym), the whole GPU suite first, then the prep-pass
  #    timing, the tile-size and byte-mirror A/Bs, and the profile of this build
  e) exec_steps=(tests smoke env:GC_PREP_TIMING=1 step:rmat26 env:GC_PREP_TIMING=
                 abl:rmat24:4:2:base=-,tile16=variants/tile16/libgcolor.so
                 ab:rmat26:3:base,c8off=GC_VALIDATE_C8:0
                 profile:rmat24) ;;
  # f: variant B's profile, the hybrid's switch point at P = 1, the tile size on the other workloads
  f) exec_steps=("profile:rmat24:--variant,B"
                 "bench:rmat24:--sharded,--multi,hybrid,--switch-below,1000000000,--steps,3,--warmup,1"
                 "bench:rmat24:--sharded,--multi,hybrid,--switch-below,262144,--steps,3,--warmup,1"
                 "bench:rmat24:--sharded,--multi,hybrid,--switch-below,16384,--steps,3,--warmup,1"
                 abl:uniform10M:6:1:base=-,tile16=variants/tile16/libgcolor.so
                 abl:mesh512:3:1:base=-,tile16=variants/tile16/libgcolor.so) ;;
  # g: the hub tests with k_propose's inlined hubs (GC_INLINE_PB), every GPU test on the build
  #    with the interleaved hub transpose, the A/Bs of the two new knobs, variant B per round
  g) exec_steps=(file:tests/test_gpu_hubs.py tests
                 ab:rmat24:6:base,inl=GC_INLINE_PB:1,abig0=GC_ASYNC_BIG:0,both=GC_INLINE_PB:1+GC_ASYNC_BIG:0
                 ab:rmat26:3:base,inl=GC_INLINE_PB:1,abig0=GC_ASYNC_BIG:0
                 brounds:rmat24) ;;
  # h: variant B's fold with compacted pending entries and the one-workgroup tail (its parity
  #    tests first), its bench and per-round cost, the tail A/B; the inline hub proposals (now
  #    on by default) through the hub and resume tests
  h) exec_steps=(file:tests/test_gpu_variant_b.py file:tests/test_gpu_hubs.py file:tests/test_gpu_resume.py
                 "bench:rmat24:--variant,B,--steps,5,--warmup,1"
                 env:AB_VARIANT=B ab:rmat24:3:base,tail0=GC_B_TAIL:0,tailbig=GC_B_TAIL_L:16384+GC_B_TAIL_E:32768
                 ab:uniform10M:4:base,tail0=GC_B_TAIL:0 env:AB_VARIANT=
                 brounds:rmat24
                 ab:rmat24:4:base,noinl=GC_INLINE_PB:0) ;;
  # i: variant B with the eviction watch and the fused pass (parity first), its A/Bs and per-round
  #    cost; the N>1 default (hybrid, strong scaling) rehearsed as two ranks on this one GPU
  i) exec_steps=(file:tests/test_gpu_variant_b.py
                 env:AB_VARIANT=B ab:rmat24:3:base,unfused=GC_B_FUSED:0,tail=GC_B_TAIL:1
                 ab:uniform10M:4:base,unfused=GC_B_FUSED:0 env:AB_VARIANT=
                 brounds:rmat24
                 "torchrun:2:--steps,2,--warmup,1,--no-north-star") ;;
  # j: validation from the low parts (symmetric graphs), its A/B on the step; variant B's tail
  #    with small caps and the per-round cost of the two-launch passes with the eviction watch
  j) exec_steps=(file:tests/test_gpu_resume.py file:tests/test_gpu_variant_b.py
                 ab:rmat26:3:base,nohalf=GC_VALIDATE_HALF:0 ab:rmat24:5:base,nohalf=GC_VALIDATE_HALF:0
                 env:AB_VARIANT=B
                 ab:rmat24:3:base,tail256=GC_B_TAIL:1+GC_B_TAIL_L:256+GC_B_TAIL_H:0+GC_B_TAIL_E:512,tail64=GC_B_TAIL:1+GC_B_TAIL_L:64+GC_B_TAIL_H:0+GC_B_TAIL_E:128
                 env:AB_VARIANT= brounds:rmat24) ;;
  # k: variant B's asynchronous fold over the compacted entries: parity, A/Bs, per-round cost
  k) exec_steps=(file:tests/test_gpu_variant_b.py
                 env:AB_VARIANT=B
                 ab:rmat24:3:base,async=GC_B_ASYNC:1,async0=GC_B_ASYNC:1+GC_B_ASYNC_K:0,async2=GC_B_ASYNC:1+GC_B_ASYNC_K:2
                 ab:uniform10M:4:base,async=GC_B_ASYNC:1
                 env:AB_VARIANT= env:GC_B_ASYNC=1 brounds:rmat24) ;;
  # l: variant B's asynchronous fold on by default (hub graphs, K = 0), the fold tail removed,
  #    long hub-list pushes flattened over the grid, the hlow-sort and async-grid knobs: every
  #    GPU test (the hub and variant B files first), smoke, then the A/Bs of the new defaults and
  #    knobs (variant B: async off / 1 / 4 workgroups per CU, the push against round 3's
  #    workgroup per winner; variant A: hlow rows unsorted) and variant B per round
  l) exec_steps=(file:tests/test_gpu_hubs.py file:tests/test_gpu_variant_b.py tests smoke
                 env:AB_VARIANT=B
                 ab:rmat24:3:base,off=GC_B_ASYNC:0,bpc1=GC_B_ASYNC_BPC:1,bpc4=GC_B_ASYNC_BPC:4
                 abl:rmat24:3:2:base=-,pushwg=variants/pushwg/libgcolor.so
                 ab:uniform10M:4:base,on=GC_B_ASYNC:1
                 env:AB_VARIANT=
                 ab:rmat24:5:base,nosort=GC_HLOW_SORT:0 ab:rmat26:3:base,nosort=GC_HLOW_SORT:0
                 brounds:rmat24 profile:rmat24 "profile:rmat24:--variant,B") ;;
  # m: the round's final build (variant B's asynchronous fold at 4 workgroups per CU): the hub and
  #    variant B tests, smoke, the profiles of THIS build (A and B on R-MAT-24, A on R-MAT-26:
  #    profiles/pmc), the default bench line, then the async grid beyond 4 (for the record)
  m) exec_steps=(file:tests/test_gpu_hubs.py file:tests/test_gpu_variant_b.py smoke
                 profile:rmat24 "profile:rmat24:--variant,B" profile:rmat26
                 "bench:rmat24"
                 env:AB_VARIANT=B ab:rmat24:3:base,bpc6=GC_B_ASYNC_BPC:6,bpc8=GC_B_ASYNC_BPC:8 env:AB_VARIANT=) ;;
  # n: the final build again (no rebuild): variant B against the oracle at R-MAT-20 (asynchronous
  #    fold and passes), variant A's per-round cost, variant B's K at 4 workgroups per CU
  n) exec_steps=(file:tests/test_gpu_variant_b.py:rmat20 rounds:rmat24
                 env:AB_VARIANT=B ab:rmat24:3:base,k1=GC_B_ASYNC_K:1 env:AB_VARIANT=) ;;
  # o: the final build with variant B's per-class timing (KTimer shared with the one-GPU engine):
  #    every GPU test, smoke, the profiles of THIS build, the variant B bench line (its roofline)
  o) exec_steps=(file:tests/test_gpu_variant_b.py tests smoke
                 profile:rmat24 "profile:rmat24:--variant,B" profile:rmat26) ;;
  # p: the final build's per-graph phases (GC_PREP_TIMING) on R-MAT-24 and R-MAT-26 (no rebuild)
  p) exec_steps=(env:GC_PREP_TIMING=1 step:rmat24 step:rmat26 env:GC_PREP_TIMING=) ;;
  # q: the hub low rows sorted in LDS: the order check on both sort paths, every GPU test, the
  #    A/B against rocPRIM's segmented sort, the phase times
  q) exec_steps=(file:tests/test_gpu_hubs.py:hlow_rows_sorted tests smoke
                 ab:rmat24:5:base,rocprim=GC_HLOW_LDS:0 ab:rmat26:3:base,rocprim=GC_HLOW_LDS:0
                 env:GC_PREP_TIMING=1 step:rmat26 env:GC_PREP_TIMING=) ;;
  # r: the hybrid's switch point on R-MAT-26 at P = 1 (no rebuild)
  r) exec_steps=("bench:rmat26:--sharded,--multi,hybrid,--switch-below,1000000000,--steps,2,--warmup,1,--no-north-star"
                 "bench:rmat26:--sharded,--multi,hybrid,--steps,2,--warmup,1,--no-north-star"
                 "bench:rmat26:--sharded,--multi,hybrid,--switch-below,65536,--steps,2,--warmup,1,--no-north-star") ;;
  # s: the hybrid's switch after the frontier peak (host change only): R-MAT-26 and R-MAT-24 at
  #    P = 1, the shard tests, and the N = 2 default again as two ranks over gloo on this GPU
  s) exec_steps=("bench:rmat26:--sharded,--multi,hybrid,--steps,2,--warmup,1,--no-north-star"
                 "bench:rmat24:--sharded,--multi,hybrid,--steps,3,--warmup,1,--no-north-star"
                 file:tests/test_gpu_resume.py:hybrid file:tests/test_shard_gpu.py
                 "torchrun:2:--steps,2,--warmup,1,--no-north-star") ;;
  # t: the final build on the other configurations (C2 uniform 10M, C4 mesh 512^3, C5 R-MAT-28),
  #    variant A and C2 variant B, for the record (no rebuild)
  t) exec_steps=("bench:uniform10M:--no-north-star,--no-cpu-baseline,--no-end-to-end"
                 "bench:mesh512:--no-north-star,--no-cpu-baseline,--no-end-to-end,--steps,5"
                 "bench:rmat28:--no-north-star,--no-cpu-baseline,--no-end-to-end,--steps,3,--warmup,1"
                 "bench:uniform10M:--variant,B,--no-north-star,--no-cpu-baseline,--no-end-to-end") ;;
  # u: the default bench line with its phase lines (the round-end command), then C5 R-MAT-28
  u) exec_steps=(bench:rmat24
                 "bench:rmat28:--no-north-star,--no-cpu-baseline,--no-end-to-end,--steps,2,--warmup,1") ;;
  # v: the hub memory check from the actual hlow size: the full-size tests first (R-MAT-28 now
  #    with hubs), every GPU test, smoke, C5's bench step, then the profiles of this build
  v) exec_steps=(file:tests/test_gpu_fullsize.py tests smoke
                 "bench:rmat28:--no-north-star,--no-cpu-baseline,--no-end-to-end,--steps,3,--warmup,1"
                 profile:rmat24 "profile:rmat24:--variant,B" profile:rmat26) ;;
  # w: C5's hybrid at P = 1 (R-MAT-28 as one shard, then the engine; no rebuild)
  w) exec_steps=("bench:rmat28:--sharded,--multi,hybrid,--steps,2,--warmup,1,--no-north-star") ;;
  *) echo "usage: $0 a|b|c|d|e|f|g|h|i|j|k|l|m|n|o|p|q|r|s|t|u|v|w" >&2; exit 2 ;;
esac
bash tools/gpu_session.sh "r04$1" "${exec_steps[@]}"
