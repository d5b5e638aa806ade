#!/bin/bash
# Round 5's GPU sessions, one gpurun call each (<= 1200 s):
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash tools/gpu_plan_r05.sh a
#   a: FETCH_SIZE / WRITE_SIZE per op of the engine's access patterns, then
#      C5's one-GPU step with the colouring's set-up phases and every large hipMalloc / hipFree
#      timed (~1.36 s of R-MAT-28's step is outside the rounds), R-MAT-26 beside it
set -uo pipefail
cd "$(dirname "$0")/.."
case ${1:-} in
  a) exec_steps=(calib env:GC_PREP_TIMING=1 env:GC_ALLOC_TRACE=1 step:rmat28 step:rmat26 env:GC_PREP_TIMING= env:GC_ALLOC_TRACE=) ;;
  # b: the allocator's idle cap at half of HBM (no ~3 s hipMalloc stall after a step's frees), the
  #    range validation, the stage-overflow halt, exact launch counts, the RCCL one-rank group and
  #    bench.py --gpus 2 (new tests first), every GPU test, smoke, C5's step and the default line
  b) exec_steps=("file:tests/test_gpu_resume.py:validate_range~or~list_overflow"
                 "file:tests/test_shard_gpu.py:one_rank_rccl" file:tests/test_bench_gpu.py tests smoke
                 "bench:rmat28:--no-north-star,--no-cpu-baseline,--no-end-to-end,--steps,3,--warmup,1"
                 bench:rmat24) ;;
  # c: the numpy replica of the device R-MAT generator (the full-size fixtures are built from it)
  #    against the device graph; the floor of a small round: six kernel launches against one
  #    resident launch confined to one XCD, or spanning the device (tools/ubench/round_floor.hip)
  c) exec_steps=("py:tools/check_rmat_replica.py:12,16,20" ubench:round_floor:200) ;;
  # d: the asynchronous kernels' grids capped at the measured residency (a probe launch of the
  #    same kernel): the variant B and hub tests, then the grid A/Bs (variant B 4 / 6 / 8 per CU,
  #    8 now meaning the measured maximum; variant A 2 / 4 / 8)
  d) exec_steps=("file:tests/test_gpu_variant_b.py:residency~or~rmat20" file:tests/test_gpu_hubs.py
                 env:AB_VARIANT=B ab:rmat24:3:base,bpc6=GC_B_ASYNC_BPC:6,bpc8=GC_B_ASYNC_BPC:8 env:AB_VARIANT=
                 ab:rmat24:4:base,bpc4=GC_ASYNC_BPC:4,bpc8=GC_ASYNC_BPC:8) ;;
  # e: the asynchronous kernels at 2..8 workgroups per CU requested (measured residency, give-ups)
  e) exec_steps=("py:tools/b_grid_probe.py:20") ;;
  # f: the hub threshold against the whole step (the hub index's build grows with the hub
  #    entries: R-MAT-28 hin count 70 + fill 100 + hlow sort 35 ms at 512), and variant B's
  #    fold grid 4 vs 6 per CU
  f) exec_steps=(ab:rmat24:5:base,t384=GC_HUB_T:384,t1024=GC_HUB_T:1024,t2048=GC_HUB_T:2048
                 ab:rmat26:3:base,t1024=GC_HUB_T:1024,t2048=GC_HUB_T:2048
                 ab:rmat28:2:base,t1024=GC_HUB_T:1024,t2048=GC_HUB_T:2048
                 env:AB_VARIANT=B ab:rmat24:4:base,bpc6=GC_B_ASYNC_BPC:6 env:AB_VARIANT=) ;;
  # g: hub flags from the rank partition (the hub transpose's count streams them instead of a
  #    gathered hub bit per entry): the hub tests, every GPU test, the phase times of R-MAT-28 /
  #    R-MAT-26, and the A/B against the gathers (GC_HUB_FLAGS=0)
  g) exec_steps=(file:tests/test_gpu_hubs.py tests env:GC_PREP_TIMING=1 step:rmat28 step:rmat26 env:GC_PREP_TIMING=
                 ab:rmat26:3:base,gather=GC_HUB_FLAGS:0 ab:rmat24:5:base,gather=GC_HUB_FLAGS:0
                 ab:rmat28:2:base,gather=GC_HUB_FLAGS:0) ;;
  # h: variant B's 7-per-CU cliff under a 10x longer give-up budget (slow progress or a stall?)
  h) exec_steps=("py:tools/b_cliff_probe.py") ;;
  # i: the R-MAT-27 fixture of the multi-core restatement (minutes on 16 threads, heartbeats),
  #    then every GPU test, the phase times and the hub-flag A/Bs of session g
  i) exec_steps=("py:tools/make_rmat27_omp_fixture.py:gpurun_out/r05i/rmat_omp_s27.json" tests) ;;
  # j: the phase times with the partition's hub flags, the A/B against the gathers, variant B's cliff
  j) exec_steps=(file:tests/test_gpu_fullsize.py:rmat27_engine env:GC_PREP_TIMING=1 step:rmat28 step:rmat26 step:rmat24 env:GC_PREP_TIMING=
                 ab:rmat26:3:base,gather=GC_HUB_FLAGS:0 ab:rmat24:5:base,gather=GC_HUB_FLAGS:0
                 ab:rmat28:2:base,gather=GC_HUB_FLAGS:0 "py:tools/b_cliff_probe.py") ;;
  # k: the rocprofv3 summaries of THIS build (kernel trace + FETCH / WRITE passes -> profiles/pmc),
  #    the five single-GPU workloads the bench lines read them for
  k) exec_steps=(profile:rmat24 "profile:rmat24:--variant,B" profile:rmat26) ;;
  k2) exec_steps=(profile:mesh512 profile:uniform10M) ;;
  k3) exec_steps=(profile:mesh512) ;;
  # l: the N > 1 step rehearsed at scale: bench.py --gpus 2 (it starts the two ranks itself) on
  #    R-MAT-26, both ranks on this box's one GPU over gloo
  l) exec_steps=(env:GC_BENCH_BACKEND=gloo env:GC_BENCH_DEVICE=0
                 "bench:rmat24:--gpus,2,--steps,2,--warmup,1" env:GC_BENCH_BACKEND= env:GC_BENCH_DEVICE=
                 "bench:rmat26:--sharded,--steps,2,--warmup,1" "bench:rmat28:--sharded,--steps,2,--warmup,1") ;;
  # m: the partition's hub flags at the flag-free kernel's occupancy (bit masks: 95 VGPRs, 5 waves
  #    per SIMD, was 102 / 4): hub + parity tests, the A/B against the gathers again
  m) exec_steps=(file:tests/test_gpu_hubs.py file:tests/test_gpu_parity.py
                 ab:rmat26:3:base,gather=GC_HUB_FLAGS:0 ab:rmat24:5:base,gather=GC_HUB_FLAGS:0
                 ab:rmat28:2:base,gather=GC_HUB_FLAGS:0) ;;
  # n: variant B's stall at 7 per CU with an agent-scope acquire (L2 invalidate) in the fold's idle
  #    path (variants/bidle: -DGC_B_IDLE_ACQ=1): stale lines kept alive by the pollers?
  n) exec_steps=(env:GC_LIB_PATH=variants/bidle/libgcolor.so "py:tools/b_cliff_probe.py" env:GC_LIB_PATH=
                 env:AB_VARIANT=B "abl:rmat24:3:2:base=-,bidle=variants/bidle/libgcolor.so" env:AB_VARIANT=
                 "abl:rmat24:4:2:base=-,aidle=variants/abidle/libgcolor.so" brounds:rmat24) ;;
  # o: variant B's fold, per round: the slowest wave's time, passes and heavy-row time
  #    (variants/bprof: -DGC_B_PROF=1) on R-MAT-24
  o) exec_steps=(env:GC_LIB_PATH=variants/bprof/libgcolor.so env:GC_B_PROF_OUT=gpurun_out/r05o/bprof_rmat24.txt
                 "py:tools/b_round_cost.py:run,rmat24,gpurun_out/r05o/records_rmat24.json,1" env:GC_LIB_PATH= env:GC_B_PROF_OUT=) ;;
  # p: the fold's resident form (b_async_resident: a wave's last <= 64 items with their entries in
  #    LDS): variant B parity (golden, oracle, C3 full size), the A/B against GC_B_RESIDENT=0, the
  #    per-round profile again
  p) exec_steps=(file:tests/test_gpu_variant_b.py "file:tests/test_gpu_fullsize.py:c3" file:tests/test_gpu_parity.py
                 env:AB_VARIANT=B ab:rmat24:4:base,nores=GC_B_RESIDENT:0,k1=GC_B_ASYNC_K:1 env:AB_VARIANT=
                 env:GC_LIB_PATH=variants/bprof/libgcolor.so env:GC_B_PROF_OUT=gpurun_out/r05p/bprof_rmat24.txt
                 "py:tools/b_round_cost.py:run,rmat24,gpurun_out/r05p/records_rmat24.json,1" env:GC_LIB_PATH= env:GC_B_PROF_OUT=) ;;
  # q: watched admission entries (a full rescan only when the smallest pending entry settles, or
  #    every GC_B_WATCH-th pass; profiles/r05/p: 21.8 G entries scanned per R-MAT-24 colouring):
  #    parity, the A/B over GC_B_WATCH, the per-round profile
  q) exec_steps=(file:tests/test_gpu_variant_b.py "file:tests/test_gpu_fullsize.py:c3 and B" file:tests/test_gpu_parity.py
                 env:AB_VARIANT=B ab:rmat24:4:base,w0=GC_B_WATCH:0,w4=GC_B_WATCH:4,w32=GC_B_WATCH:32 env:AB_VARIANT=
                 env:GC_LIB_PATH=variants/bprof/libgcolor.so env:GC_B_PROF_OUT=gpurun_out/r05q/bprof_rmat24.txt
                 "py:tools/b_round_cost.py:run,rmat24,gpurun_out/r05q/records_rmat24.json,1" env:GC_LIB_PATH= env:GC_B_PROF_OUT=) ;;
  # r: the rank partition's fourth class (higher degree split by position: variant B's admission
  #    range is the earlier entries, its eviction range the later ones -- about half of each
  #    scan, R-MAT-20 oracle count): every GPU test, variant B's A/B against the previous
  #    build (variants/r05q), variant A's step, the per-round profile
  r) exec_steps=(file:tests/test_gpu_parity.py file:tests/test_gpu_variant_b.py "file:tests/test_gpu_fullsize.py:c3" tests
                 env:AB_VARIANT=B "abl:rmat24:3:2:base=-,prev=variants/r05q/libgcolor.so" env:AB_VARIANT=
                 "abl:rmat24:3:2:base=-,prev=variants/r05q/libgcolor.so"
                 env:GC_LIB_PATH=variants/bprof/libgcolor.so env:GC_B_PROF_OUT=gpurun_out/r05r/bprof_rmat24.txt
                 "py:tools/b_round_cost.py:run,rmat24,gpurun_out/r05r/records_rmat24.json,1" env:GC_LIB_PATH= env:GC_B_PROF_OUT=) ;;
  # s: variant B's fold knobs on the split partition: the watch period, the resident form, the
  #    grid (4 / 6 per CU)
  s) exec_steps=(env:AB_VARIANT=B
                 ab:rmat24:4:base,w16=GC_B_WATCH:16,w32=GC_B_WATCH:32,w64=GC_B_WATCH:64,nores=GC_B_RESIDENT:0,bpc6=GC_B_ASYNC_BPC:6
                 ab:rmat26:2:base,w32=GC_B_WATCH:32,bpc6=GC_B_ASYNC_BPC:6 env:AB_VARIANT=) ;;
  # t: variant B with pushed forbidden-colour bitmaps for more vertices (every uncoloured vertex
  #    proposes every round: rows of degree 64-512 are re-read ~13 times, R-MAT-20 oracle count)
  t) exec_steps=(env:AB_VARIANT=B ab:rmat24:3:base,t256=GC_HUB_T:256,t128=GC_HUB_T:128,t64=GC_HUB_T:64 env:AB_VARIANT=) ;;
  # u: variant A's asynchronous JP with held lights (GC_A_WATCH): parity with it on, the A/Bs
  u) exec_steps=(env:GC_A_WATCH=8 file:tests/test_gpu_parity.py file:tests/test_gpu_hubs.py "file:tests/test_gpu_fullsize.py:c3 and A"
                 env:GC_A_WATCH= ab:rmat24:4:base,aw4=GC_A_WATCH:4,aw8=GC_A_WATCH:8,aw32=GC_A_WATCH:32
                 ab:rmat26:3:base,aw8=GC_A_WATCH:8,aw32=GC_A_WATCH:32) ;;
  # v: where the N > 1 step's creation goes (R-MAT-28 one-rank RCCL: create 2046 ms against 159 at
  #    N = 1): gc_shard_create's phases and the allocator's large blocks
  v) exec_steps=(env:GC_PREP_TIMING=1 env:GC_ALLOC_TRACE=1 "bench:rmat28:--sharded,--steps,1,--warmup,1"
                 "bench:rmat26:--sharded,--steps,1,--warmup,1" env:GC_PREP_TIMING= env:GC_ALLOC_TRACE=) ;;
  # w: a shard's in-rows entry-parallel over the tiling (k_filt_count / k_filt_fill): the shard,
  #    resume and multi-GPU bench tests, then session v's creation phases again
  w) exec_steps=(file:tests/test_shard_gpu.py file:tests/test_gpu_resume.py file:tests/test_bench_gpu.py
                 "file:tests/test_gpu_fullsize.py:rmat27" file:tests/test_xl_gpu.py
                 env:GC_PREP_TIMING=1 "bench:rmat28:--sharded,--steps,1,--warmup,1"
                 "bench:rmat26:--sharded,--steps,1,--warmup,1" env:GC_PREP_TIMING=) ;;
  # x: the allocator parking all but 48 GB (the multi-GPU step's stalls), R-MAT-28 / 26 sharded
  #    and one-GPU, and the gloo two-rank rehearsal on R-MAT-26
  x) exec_steps=(env:GC_PREP_TIMING=1 env:GC_ALLOC_TRACE=1 "bench:rmat28:--sharded,--steps,2,--warmup,1"
                 env:GC_PREP_TIMING= env:GC_ALLOC_TRACE= "bench:rmat26:--sharded,--steps,2,--warmup,1"
                 "bench:rmat28:--no-north-star,--no-cpu-baseline,--no-end-to-end,--steps,3,--warmup,1"
                 env:GC_BENCH_BACKEND=gloo env:GC_BENCH_DEVICE=0 "bench:rmat26:--gpus,2,--steps,1,--warmup,1"
                 env:GC_BENCH_BACKEND= env:GC_BENCH_DEVICE=) ;;
  # y: variant B's round wait through a kernel-written snapshot (no copy-engine blit, no memset a
  #    round): parity, the A/B against GC_SNAP_COPY=1
  y) exec_steps=(file:tests/test_gpu_variant_b.py "file:tests/test_gpu_fullsize.py:c3 and B"
                 env:AB_VARIANT=B ab:rmat24:4:base,blit=GC_SNAP_COPY:1 env:AB_VARIANT=) ;;
  # z: a refused admission reads no more of its entries (GC_B_REFSKIP): parity, the A/B
  z) exec_steps=(file:tests/test_gpu_variant_b.py "file:tests/test_gpu_fullsize.py:c3 and B" file:tests/test_gpu_parity.py
                 env:AB_VARIANT=B ab:rmat24:4:base,noskip=GC_B_REFSKIP:0 ab:rmat26:2:base,noskip=GC_B_REFSKIP:0 env:AB_VARIANT=) ;;
  # aa: ascending eviction ranges (a cursor and windows, no kept list): variant B parity (golden,
  #     randomized directed rows -- the kept-list form --, R-MAT and C3 -- the ascending form),
  #     every GPU test, the A/B against GC_B_EVASC=0, the per-round profile
  aa) exec_steps=(file:tests/test_gpu_variant_b.py "file:tests/test_gpu_fullsize.py:c3" file:tests/test_gpu_parity.py tests
                  env:AB_VARIANT=B ab:rmat24:4:base,noasc=GC_B_EVASC:0 ab:rmat26:2:base,noasc=GC_B_EVASC:0 env:AB_VARIANT=) ;;
  # ab: the per-round fold profile with and without the ascending eviction ranges
  ab) exec_steps=(env:GC_LIB_PATH=variants/bprof/libgcolor.so env:GC_B_PROF_OUT=gpurun_out/r05ab/bprof_asc.txt
                  "py:tools/b_round_cost.py:run,rmat24,gpurun_out/r05ab/records_asc.json,1"
                  env:GC_B_EVASC=0 env:GC_B_PROF_OUT=gpurun_out/r05ab/bprof_noasc.txt
                  "py:tools/b_round_cost.py:run,rmat24,gpurun_out/r05ab/records_noasc.json,1"
                  env:GC_B_EVASC= env:GC_LIB_PATH= env:GC_B_PROF_OUT=) ;;
  # ac: variant A's rounds by frontier class (where R-MAT-24's 130 ms of rounds go), and R-MAT-26
  ac) exec_steps=(rounds:rmat24 rounds:rmat26) ;;
  # fin: the final build: every GPU test, smoke, the default bench line (R-MAT-24 + north star + CPU
  #      baseline, traffic from profiles/pmc), C5 on one GPU, variant B, C4 and C2
  fin) exec_steps=(tests smoke bench:rmat24 "bench:rmat28:--no-north-star,--no-cpu-baseline,--no-end-to-end,--steps,3,--warmup,1"
                   "bench:rmat24:--variant,B,--no-north-star,--no-cpu-baseline,--no-end-to-end"
                   "bench:mesh512:--no-cpu-baseline,--no-end-to-end" "bench:uniform10M:--no-cpu-baseline,--no-end-to-end") ;;
  # ad: variant B's pipelined rounds (the commit decides; round r + 1 in flight while the host reads
  #     round r): variant B parity (incl. forced give-ups and the passes-only path), the A/B
  ad) exec_steps=(file:tests/test_gpu_variant_b.py "file:tests/test_gpu_fullsize.py:c3 and B" file:tests/test_gpu_resume.py
                  env:AB_VARIANT=B ab:rmat24:4:base,nopipe=GC_B_PIPE:0 ab:rmat26:2:base,nopipe=GC_B_PIPE:0
                  ab:uniform10M:4:base,nopipe=GC_B_PIPE:0 env:AB_VARIANT=) ;;
  # ae: where variant B's round goes with and without pipelining (kernel traces, per-round wall)
  ae) exec_steps=(brounds:rmat24 env:GC_B_PIPE=0 brounds:rmat24 env:GC_B_PIPE=) ;;
  # af: variant A's launch-shape knobs re-swept on today's engine (most were set in round 2)
  af) exec_steps=("ab:rmat24:4:base,c512=GC_GRID_C:512,c1024=GC_GRID_C:1024,p512=GC_GRID_P:512,p2048=GC_GRID_P:2048,cb512=GC_GRID_CB:512,cb2048=GC_GRID_CB:2048,br1024=GC_BIGROW:1024,br4096=GC_BIGROW:4096"
                  "ab:rmat24:4:base,b2=GC_BATCH_MAX:2,b8=GC_BATCH_MAX:8,abpc3=GC_ASYNC_BPC:3,s128=GC_GRID_S:128,s512=GC_GRID_S:512,ps256=GC_GRID_PS:256,ps1024=GC_GRID_PS:1024,r512=GC_GRID_R:512,r2048=GC_GRID_R:2048") ;;
  # ag: the rocprofv3 summaries of C5 (R-MAT-28 on one GPU) for its bench line's traffic
  ag) exec_steps=("profile:rmat28:--no-north-star,--no-cpu-baseline,--no-end-to-end") ;;
  # ah: entries in flight per lane on today's engine (GC_SLOTS 1 / 2 / 4: the light kernels' edge
  #     chunks; GC_CSLOTS 4: the commit's claims), where the rounds are bandwidth-bound (R-MAT-26/28)
  ah) exec_steps=("abl:rmat26:3:2:base=-,s4=variants/s4/libgcolor.so,cs4=variants/cs4/libgcolor.so,s1=variants/s1/libgcolor.so"
                  "abl:rmat24:3:2:base=-,s4=variants/s4/libgcolor.so,cs4=variants/cs4/libgcolor.so") ;;
  # ai: bench.py --gpus 4 and --gpus 8 end to end (it starts the ranks itself), every rank on this
  #     box's one GPU over gloo: the 4- and 8-rank paths of the driver's scaling runs, not timings
  ai) exec_steps=(env:GC_BENCH_BACKEND=gloo env:GC_BENCH_DEVICE=0
                  "bench:rmat20:--gpus,4,--steps,1,--warmup,1" "bench:rmat20:--gpus,8,--steps,1,--warmup,1"
                  env:GC_BENCH_BACKEND= env:GC_BENCH_DEVICE=) ;;
  # aj: variant B's fold, first scans against rescans per round (variants/bprof: -DGC_B_PROF=1)
  aj) exec_steps=(env:GC_LIB_PATH=variants/bprof/libgcolor.so env:GC_B_PROF_OUT=gpurun_out/r05aj/bprof_rmat24.txt
                  "py:tools/b_round_cost.py:run,rmat24,gpurun_out/r05aj/records_rmat24.json,1" env:GC_LIB_PATH= env:GC_B_PROF_OUT=) ;;
  # ak: admission cursors (a window of pending entries from a cursor between full rescans, instead
  #     of a full rescan whenever the smallest pending entry settles): variant B parity, the A/B
  #     against the previous build (variants/prev), the watch period
  ak) exec_steps=(file:tests/test_gpu_variant_b.py "file:tests/test_gpu_fullsize.py:c3 and B" file:tests/test_gpu_parity.py
                  env:AB_VARIANT=B "abl:rmat24:3:2:base=-,prev=variants/prev/libgcolor.so" "abl:rmat26:2:2:base=-,prev=variants/prev/libgcolor.so"
                  ab:rmat24:3:base,w4=GC_B_WATCH:4,w32=GC_B_WATCH:32 env:AB_VARIANT=) ;;
  al) exec_steps=(file:tests/test_gpu_variant_b.py env:AB_VARIANT=B
                  "ab:rmat24:3:base,w4=GC_B_WATCH:4,w2=GC_B_WATCH:2,w4a32=GC_B_WATCH:4+GC_B_AWIN:32,w4a8=GC_B_WATCH:4+GC_B_AWIN:8,w8a32=GC_B_AWIN:32,w8a64=GC_B_AWIN:64"
                  "ab:rmat26:2:base,w4=GC_B_WATCH:4,w4a32=GC_B_WATCH:4+GC_B_AWIN:32,w8a32=GC_B_AWIN:32"
                  env:AB_VARIANT=) ;;
  am) exec_steps=(env:AB_VARIANT=B
                  "ab:rmat24:3:base,a8=GC_B_AWIN:8,a4=GC_B_AWIN:4,w16a8=GC_B_WATCH:16+GC_B_AWIN:8,w16a4=GC_B_WATCH:16+GC_B_AWIN:4,w4a4=GC_B_WATCH:4+GC_B_AWIN:4"
                  "ab:rmat26:2:base,a8=GC_B_AWIN:8,a4=GC_B_AWIN:4,w16a8=GC_B_WATCH:16+GC_B_AWIN:8,w4a8=GC_B_WATCH:4+GC_B_AWIN:8"
                  env:AB_VARIANT=) ;;
  an) exec_steps=(file:tests/test_gpu_variant_b.py "file:tests/test_gpu_fullsize.py:c3 and B"
                  profile:rmat24 "profile:rmat24:--variant,B" profile:rmat26) ;;
  ao) exec_steps=(profile:mesh512 profile:uniform10M "profile:rmat28:--no-north-star,--no-cpu-baseline,--no-end-to-end") ;;
  # ap: the fold's scanned entries with the admission cursors (variants/bprof: -DGC_B_PROF=1 with the
  #     first-scan / admission-rescan / eviction-rescan split), and with them off (GC_B_WATCH=0)
  ap) exec_steps=(env:GC_LIB_PATH=variants/bprof/libgcolor.so env:GC_B_PROF_OUT=gpurun_out/r05ap/bprof_rmat24.txt
                  "py:tools/b_round_cost.py:run,rmat24,gpurun_out/r05ap/records_rmat24.json,1"
                  env:GC_B_WATCH=0 env:GC_B_PROF_OUT=gpurun_out/r05ap/bprof_rmat24_w0.txt
                  "py:tools/b_round_cost.py:run,rmat24,gpurun_out/r05ap/records_rmat24_w0.json,1"
                  env:GC_LIB_PATH= env:GC_B_PROF_OUT= env:GC_B_WATCH=) ;;
  # aq: the cursor entry checked before the window (GC_B_HOLD): variant B parity, the A/B
  aq) exec_steps=(file:tests/test_gpu_variant_b.py "file:tests/test_gpu_fullsize.py:c3 and B" env:AB_VARIANT=B
                  "ab:rmat24:3:base,hold0=GC_B_HOLD:0,a16=GC_B_AWIN:16,w8a16=GC_B_WATCH:8+GC_B_AWIN:16"
                  "ab:rmat26:2:base,hold0=GC_B_HOLD:0,a16=GC_B_AWIN:16" env:AB_VARIANT=) ;;
  # ar: the N > 1 bench paths on the final build (every rank on this box's one GPU over gloo)
  ar) exec_steps=(env:GC_BENCH_BACKEND=gloo env:GC_BENCH_DEVICE=0
                  "bench:rmat24:--gpus,2,--steps,2,--warmup,1" "bench:rmat20:--gpus,4,--steps,1,--warmup,1"
                  "bench:rmat20:--gpus,8,--steps,1,--warmup,1" env:GC_BENCH_BACKEND= env:GC_BENCH_DEVICE=) ;;
  # as: variant B at R-MAT-26 on the final build (trace + PMC passes)
  as) exec_steps=("profile:rmat26:--variant,B,--no-north-star,--no-cpu-baseline,--no-end-to-end") ;;
  # at: the fold's resident form capped at 1024 / 2048 entries per wave (compile-time; LDS: 5 / 3
  #     workgroups per CU instead of 4), and 1024 with 5 workgroups per CU (GC_B_ASYNC_BPC=5)
  at) exec_steps=(env:AB_VARIANT=B
                  "abl:rmat24:3:2:base=-,r1024=variants/r1024/libgcolor.so,r2048=variants/r2048/libgcolor.so"
                  env:GC_B_ASYNC_BPC=5 "abl:rmat24:3:2:base=-,r1024b5=variants/r1024/libgcolor.so"
                  "abl:rmat26:2:2:base=-,r1024b5=variants/r1024/libgcolor.so" env:GC_B_ASYNC_BPC=
                  "abl:rmat26:2:2:base=-,r1024=variants/r1024/libgcolor.so" env:AB_VARIANT=) ;;
  au) exec_steps=(profile:mesh512 profile:uniform10M "profile:rmat28:--no-north-star,--no-cpu-baseline,--no-end-to-end"
                  "profile:rmat26:--variant,B,--no-north-star,--no-cpu-baseline,--no-end-to-end") ;;
  # av: 6 workgroups per CU for the fold (variants/w6: amdgpu_waves_per_eu(6), 80 VGPRs with 28 B of
  #     scratch, resident cap 768; variants/c768: the cap alone) -- for the next round, not the build
  av) exec_steps=(env:AB_VARIANT=B env:GC_B_ASYNC_BPC=6
                  "abl:rmat24:3:2:base=-,w6=variants/w6/libgcolor.so,c768=variants/c768/libgcolor.so"
                  "abl:rmat26:2:2:base=-,w6=variants/w6/libgcolor.so" env:GC_B_ASYNC_BPC= env:AB_VARIANT=) ;;
  aw) exec_steps=(file:tests/test_gpu_variant_b.py "file:tests/test_gpu_fullsize.py:c3 and B"
                  profile:rmat24 "profile:rmat24:--variant,B" profile:rmat26
                  profile:mesh512 profile:uniform10M "profile:rmat28:--no-north-star,--no-cpu-baseline,--no-end-to-end"
                  "profile:rmat26:--variant,B,--no-north-star,--no-cpu-baseline,--no-end-to-end") ;;
  *) echo "usage: $0 a|b|...|z|aa|ab|ac|fin|ad|ae|af|ag|ah|ai|aj|ak|al|am|an|ao|ap|aq|ar|as|at|au|av|aw" >&2; exit 2 ;;
esac
bash tools/gpu_session.sh "r05$1" "${exec_steps[@]}"
