#!/bin/bash
# Round 6's GPU sessions, one gpurun call each (<= 1200 s):
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash tools/gpu_plan_r06.sh a
# (round 5's sessions: tools/gpu_plan_r05.sh; the step kinds: tools/gpu_session.sh)
set -uo pipefail
cd "$(dirname "$0")/.."
case ${1:-} in
  # a: the round-5 build's line on this box, then where k_sweep_async's time goes per round
  #    (variants/aprof: -DGC_A_PROF=1 -- light phase, wait for the last light, hub phase, passes)
  #    on R-MAT-24 and R-MAT-26
  a) exec_steps=("bench:rmat24:--no-north-star,--no-cpu-baseline,--no-end-to-end"
                 env:GC_LIB_PATH=variants/aprof/libgcolor.so env:GC_A_PROF_OUT=gpurun_out/r06a/aprof_rmat24.txt
                 "py:tools/round_cost.py:run,rmat24,gpurun_out/r06a/records_rmat24.json,1"
                 env:GC_A_PROF_OUT=gpurun_out/r06a/aprof_rmat26.txt
                 "py:tools/round_cost.py:run,rmat26,gpurun_out/r06a/records_rmat26.json,1"
                 env:GC_LIB_PATH= env:GC_A_PROF_OUT=) ;;
  # a2: the same with the hub scan's entries counted (scanned, longest scan, winners, entries left)
  a2) exec_steps=(env:GC_LIB_PATH=variants/aprof/libgcolor.so env:GC_A_PROF_OUT=gpurun_out/r06a2/aprof_rmat24.txt
                 "py:tools/round_cost.py:run,rmat24,gpurun_out/r06a2/records_rmat24.json,1"
                 env:GC_A_PROF_OUT=gpurun_out/r06a2/aprof_rmat26.txt
                 "py:tools/round_cost.py:run,rmat26,gpurun_out/r06a2/records_rmat26.json,1"
                 env:GC_LIB_PATH= env:GC_A_PROF_OUT=) ;;
  # b: the hub core (csrc/gc_core.hip): its parity tests, the hub settings, then the interleaved A/B
  b) exec_steps=(env:GC_CORE_DEBUG=1 "py:tools/core_probe.py" env:GC_CORE_DEBUG=
                 file:tests/test_gpu_core.py file:tests/test_gpu_hubs.py file:tests/test_gpu_parity.py
                 "ab:rmat24:3:base,nocore=GC_HUB_CORE:0" "ab:rmat26:2:base,nocore=GC_HUB_CORE:0") ;;
  # c: k_hub_core's launch times against k_sweep_async's (kernel trace of R-MAT-24, core on then off)
  c) mkdir -p gpurun_out/r06c && cd /tmp && export TMPDIR=/tmp &&
     timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/gpurun_out/r06c/trace" -o run -- \
       python3 "$GRAFT_REPO_ROOT/tools/core_probe.py" 24:512 > "$GRAFT_REPO_ROOT/gpurun_out/r06c/probe.log" 2>&1
     rc=$?; cd "$GRAFT_REPO_ROOT"; f=$(find gpurun_out/r06c/trace -name '*kernel_stats.csv' | head -1)
     [ -n "$f" ] && cp "$f" gpurun_out/r06c/kernel_stats.csv; find gpurun_out/r06c/trace -name '*kernel_trace.csv' -delete
     [ $rc -eq 0 ] || exit $rc
     GC_LIB_PATH=variants/aprof/libgcolor.so GC_A_PROF_OUT=gpurun_out/r06c/aprof_rmat24.txt timeout -k 10 300 \
       python -u tools/round_cost.py run rmat24 gpurun_out/r06c/records_rmat24.json 1 > gpurun_out/r06c/aprof.log 2>&1
     exit $? ;;
  # d: per-round kernel cost with the hub core (the default build), R-MAT-24, and with it off
  d) exec_steps=(rounds:rmat24:core env:GC_HUB_CORE=0 rounds:rmat24:nocore env:GC_HUB_CORE=) ;;
  # e: k_hub_core's phases per round (variants/aprof: load + setup, windows), R-MAT-24
  e) exec_steps=(file:tests/test_gpu_core.py env:GC_LIB_PATH=variants/aprof/libgcolor.so env:GC_A_PROF_OUT=gpurun_out/r06e/aprof_rmat24.txt
                 "py:tools/round_cost.py:run,rmat24,gpurun_out/r06e/records_rmat24.json,1" env:GC_LIB_PATH= env:GC_A_PROF_OUT=) ;;
  # f: variant B's fold at 6 / 7 / 8 workgroups per CU (variants/bwpe8: compiled for 8 waves per SIMD,
  #    resident cap 512), the state of the first give-up dumped (tools/b_stall_analyze.py)
  f) exec_steps=(env:GC_LIB_PATH=variants/bwpe8/libgcolor.so "py:tools/b_stall_probe.py:gpurun_out/r06f,20,6,7,8"
                 env:GC_LIB_PATH=) ;;
  # g: the fold compiled for 7 / 8 waves per SIMD (variants/bwpe7: 72 VGPRs, resident cap 640;
  #    bwpe8: 64 VGPRs, cap 512) against the default (6), GC_B_ASYNC_BPC=8 (each capped by its measured
  #    residency), variant B on R-MAT-24 and R-MAT-26; the default build at 6 / 7 / 8 per CU requested
  g) exec_steps=("py:tools/b_stall_probe.py:gpurun_out/r06g,20,6,7,8" env:AB_VARIANT=B env:GC_B_ASYNC_BPC=8
                 "abl:rmat24:3:2:base=-,w7=variants/bwpe7/libgcolor.so,w8=variants/bwpe8/libgcolor.so"
                 "abl:rmat26:2:2:base=-,w7=variants/bwpe7/libgcolor.so,w8=variants/bwpe8/libgcolor.so"
                 env:AB_VARIANT= env:GC_B_ASYNC_BPC=) ;;
  # h: C5's full-size fixture: R-MAT-28 coloured by the multi-core restatement on the box's 16 threads
  #    (tests/golden/rmat_omp_s28.json; heartbeat lines every 20 s)
  h) exec_steps=("pyl:tools/make_rmat27_omp_fixture.py:gpurun_out/r06h/rmat_omp_s28.json,28") ;;
  # i: a fold stopped on purpose (zero budget): the dumped state of its first give-up, R-MAT-18, for
  #    tools/b_stall_analyze.py (does every listed item wait on an earlier listed one?)
  i) exec_steps=(env:GC_ASYNC_BUDGET_US=0 "py:tools/b_stall_probe.py:gpurun_out/r06i,18,6" env:GC_ASYNC_BUDGET_US=) ;;
  # j: the full-size pins (R-MAT-24 restatement vs the single-thread oracle, R-MAT-26 vs the single-thread
  #    oracle, R-MAT-27/28 vs the restatement), then the hub threshold re-swept on the round-6 engine
  j) exec_steps=("file:tests/test_gpu_fullsize.py:against_single_thread_oracle~or~engine_against_multicore"
                 "ab:rmat24:3:base,t384=GC_HUB_T:384,t768=GC_HUB_T:768") ;;
  k) exec_steps=("file:tests/test_gpu_fullsize.py:engine_against_multicore"
                 "ab:rmat24:3:base,t384=GC_HUB_T:384,t768=GC_HUB_T:768,t1024=GC_HUB_T:1024"
                 "ab:rmat26:2:base,t768=GC_HUB_T:768,t1024=GC_HUB_T:1024,t2048=GC_HUB_T:2048") ;;
  m) exec_steps=("file:tests/test_gpu_hubs.py" "file:tests/test_gpu_parity.py" "file:tests/test_gpu_core.py"
                 "abl:rmat24:3:2:base=-,nopf=variants/nopf/libgcolor.so,ng8=variants/ng8/libgcolor.so,ng16=variants/ng16/libgcolor.so"
                 "abl:rmat26:2:2:base=-,nopf=variants/nopf/libgcolor.so,ng8=variants/ng8/libgcolor.so"
                 "file:tests/test_gpu_fullsize.py:engine_against_multicore") ;;
  n) exec_steps=("file:tests/test_gpu_hubs.py" "file:tests/test_gpu_parity.py" "file:tests/test_gpu_core.py"
                 "file:tests/test_gpu_fullsize.py:c3_rmat24_against_single_thread_oracle~or~c3_rmat24_hubs_match"
                 "abl:rmat24:3:2:base=-,nopf=variants/nopf/libgcolor.so,phb1=variants/phb1/libgcolor.so,ng8=variants/ng8/libgcolor.so,ng16=variants/ng16/libgcolor.so"
                 "abl:rmat26:2:2:base=-,nopf=variants/nopf/libgcolor.so,phb1=variants/phb1/libgcolor.so,ng8=variants/ng8/libgcolor.so"
                 "file:tests/test_gpu_fullsize.py:engine_against_multicore~or~north_star_rmat26") ;;
  l) exec_steps=("abl:rmat24:3:2:base=-,ng8=variants/ng8/libgcolor.so,ng16=variants/ng16/libgcolor.so,ng2=variants/ng2/libgcolor.so,ng8u4=variants/ng8u4/libgcolor.so"
                 "abl:rmat26:2:2:base=-,ng8=variants/ng8/libgcolor.so,ng16=variants/ng16/libgcolor.so,ng8u4=variants/ng8u4/libgcolor.so") ;;
  # o: the hub phase's words in registers with a watched blocker (GC_HUB_REG), heavy runs a lane
  #    each in k_commit / k_propose_block, the async lights' kill flags in batches: parity, then
  #    A/B against all four off (variants/old) and each of the two async changes off
  o) exec_steps=("file:tests/test_gpu_hubs.py" "file:tests/test_gpu_parity.py" "file:tests/test_gpu_core.py"
                 "file:tests/test_gpu_fullsize.py:c3_rmat24_against_single_thread_oracle~or~c3_rmat24_hubs_match"
                 "abl:rmat24:3:2:base=-,old=variants/old/libgcolor.so,noreg=variants/noreg/libgcolor.so,nodefer=variants/nodefer/libgcolor.so,nohint=variants/nohint/libgcolor.so"
                 "abl:rmat26:2:2:base=-,old=variants/old/libgcolor.so") ;;
  # p: session o's build with the hub phase's owner lanes from LDS and the kill flags raised while
  #    a wave waits: parity, then A/B on R-MAT-24 and R-MAT-26
  p) exec_steps=("file:tests/test_gpu_hubs.py" "file:tests/test_gpu_parity.py"
                 "file:tests/test_gpu_fullsize.py:c3_rmat24_against_single_thread_oracle~or~c3_rmat24_hubs_match"
                 "abl:rmat24:3:2:base=-,old=variants/old/libgcolor.so,noreg=variants/noreg/libgcolor.so,nodefer=variants/nodefer/libgcolor.so,nohoist=variants/nohoist/libgcolor.so"
                 "abl:rmat26:2:2:base=-,old=variants/old/libgcolor.so,noreg=variants/noreg/libgcolor.so,nodefer=variants/nodefer/libgcolor.so") ;;
  # q: + the async lights' words in LDS (GC_LIGHT_LDS) and check-before-mark (GC_MARK_CHECK): the
  #    parity files, then A/B against all off (variants/old) and each change off
  q) V="old=variants/old/libgcolor.so,noreg=variants/noreg/libgcolor.so,nodefer=variants/nodefer/libgcolor.so"
     V="$V,nohoist=variants/nohoist/libgcolor.so,nolds=variants/nolds/libgcolor.so,nomark=variants/nomark/libgcolor.so"
     exec_steps=("file:tests/test_gpu_hubs.py" "file:tests/test_gpu_parity.py" "file:tests/test_gpu_variant_b.py"
                 "file:tests/test_gpu_fullsize.py:c3_rmat24_against_single_thread_oracle~or~c3_rmat24_hubs_match"
                 "abl:rmat24:3:2:base=-,$V"
                 "abl:rmat26:2:1:base=-,$V") ;;
  # r: the defaults q chose (registers and batched kills off, hoist off); A/B of the hub phase in
  #    registers with / without the watched blocker, the heavy runs a lane each off, the hint off,
  #    the lights' LDS words off; then the per-round cost of the new default build
  r) V="reg=variants/reg/libgcolor.so,regnw=variants/regnw/libgcolor.so,nolanes=variants/nolanes/libgcolor.so"
     V="$V,nohint=variants/nohint/libgcolor.so,nolds=variants/nolds/libgcolor.so"
     exec_steps=("file:tests/test_gpu_hubs.py" "file:tests/test_gpu_parity.py" "file:tests/test_gpu_core.py"
                 "abl:rmat24:3:2:base=-,$V"
                 "abl:rmat26:2:1:base=-,$V"
                 rounds:rmat24) ;;
  # s: one hub per wave with all 64 lanes while the hubs fit (GC_HUB_WIDE), the hub words in
  #    registers without the watch (GC_HUB_REG) above that, the lights' LDS rows only in big rounds:
  #    parity, A/B against each off and against round 5's kernels (variants/r5), per-round cost
  s) V="nowide=variants/nowide/libgcolor.so,noreg=variants/noreg/libgcolor.so,nolds=variants/nolds/libgcolor.so"
     V="$V,r5=variants/r5/libgcolor.so"
     exec_steps=("file:tests/test_gpu_hubs.py" "file:tests/test_gpu_parity.py" "file:tests/test_gpu_core.py"
                 "file:tests/test_gpu_fullsize.py:c3_rmat24_against_single_thread_oracle~or~c3_rmat24_hubs_match"
                 "abl:rmat24:3:2:base=-,$V"
                 "abl:rmat26:2:1:base=-,$V"
                 rounds:rmat24) ;;
  # t: the hub bitmaps word-major (GC_HB_WMAJOR): parity (A, B, priorities, shards), A/B, round cost
  t) V="nowm=variants/nowm/libgcolor.so"
     exec_steps=("file:tests/test_gpu_hubs.py" "file:tests/test_gpu_parity.py" "file:tests/test_gpu_variant_b.py"
                 "file:tests/test_gpu_priority.py" "file:tests/test_shard_gpu.py"
                 "file:tests/test_gpu_fullsize.py:c3_rmat24_against_single_thread_oracle~or~c3_rmat24_hubs_match"
                 "abl:rmat24:3:3:base=-,$V"
                 "abl:rmat26:2:2:base=-,$V"
                 rounds:rmat24) ;;
  # u: + k_propose's heavy appends staged per workgroup, minimum chunk sizes in small rounds, k_commit_big
  #    four entries a thread, k_commit_big closing the round (GC_CB_CLOSE), the one-hub-per-wave slices
  #    in registers: parity (A, B, priorities, shards, resume), A/B of each, round cost
  u) V="nowm=variants/nowm/libgcolor.so,nostage=variants/nostage/libgcolor.so,vmin1=variants/vmin1/libgcolor.so"
     V="$V,nocbu=variants/nocbu/libgcolor.so,noreg=variants/noreg/libgcolor.so"
     exec_steps=("file:tests/test_gpu_hubs.py" "file:tests/test_gpu_parity.py" "file:tests/test_gpu_variant_b.py"
                 "file:tests/test_gpu_priority.py" "file:tests/test_shard_gpu.py" "file:tests/test_gpu_resume.py"
                 "file:tests/test_gpu_fullsize.py:c3_rmat24_against_single_thread_oracle~or~c3_rmat24_hubs_match"
                 "abl:rmat24:3:2:base=-,$V"
                 "ab:rmat24:3:base,nocbclose=GC_CB_CLOSE:0"
                 "abl:rmat26:2:1:base=-,$V"
                 rounds:rmat24) ;;
  # v: the defaults u chose (hub-major bitmaps, k_commit_big one entry a step, k_close kept): parity, A/B
  #    against round 5's kernels (variants/r5) on every bench workload, the word-major bitmaps again, round cost
  v) exec_steps=("file:tests/test_gpu_hubs.py" "file:tests/test_gpu_parity.py"
                 "abl:rmat24:3:2:base=-,wm=variants/wm/libgcolor.so,r5=variants/r5/libgcolor.so"
                 "abl:rmat26:2:1:base=-,r5=variants/r5/libgcolor.so"
                 "abl:uniform10M:5:1:base=-,r5=variants/r5/libgcolor.so"
                 "abl:mesh512:3:1:base=-,r5=variants/r5/libgcolor.so"
                 rounds:rmat24) ;;
  # w: + a winner's in-row and hub list as one flat walk in k_commit (GC_COMMIT_FLAT), the minimum chunk
  #    only for the unfused commit: parity, A/B, the other workloads against round 5's kernels, round cost
  w) exec_steps=("file:tests/test_gpu_hubs.py" "file:tests/test_gpu_parity.py" "file:tests/test_gpu_priority.py"
                 "abl:rmat24:3:2:base=-,noflat=variants/noflat/libgcolor.so,r5=variants/r5/libgcolor.so"
                 "abl:rmat26:2:1:base=-,noflat=variants/noflat/libgcolor.so"
                 "abl:uniform10M:5:2:base=-,r5=variants/r5/libgcolor.so"
                 "abl:mesh512:3:2:base=-,r5=variants/r5/libgcolor.so"
                 rounds:rmat24) ;;
  # x: the build w chose (no flat walk): every GPU test, smoke, the asynchronous kernels' workgroups per CU
  x) exec_steps=(tests smoke "ab:rmat24:3:base,bpc3=GC_ASYNC_BPC:3,bpc4=GC_ASYNC_BPC:4"
                 "ab:rmat26:2:base,bpc3=GC_ASYNC_BPC:3") ;;
  # y / z: rocprofv3 summaries of the final build (bench line, kernel trace, FETCH_SIZE / WRITE_SIZE passes)
  y) exec_steps=(profile:rmat24 "profile:rmat24:--variant,B") ;;
  z) exec_steps=(profile:rmat26 "ab:rmat24:3:base,t384=GC_HUB_T:384,t768=GC_HUB_T:768,t1024=GC_HUB_T:1024") ;;
  z2) exec_steps=("profile:rmat28:--no-cpu-baseline,--no-north-star,--no-variant-b") ;;  # (the CPU leg on R-MAT-28 prints nothing for > 3 min)
  # fin: the default bench line of the final build (the committed profiles/pmc summaries in use) and smoke
  fin) exec_steps=(smoke bench:rmat24) ;;
  # ab2: minimum chunks for the round's first sweep (k_resolve) and 32 for propose / commit (variants built
  #    from a scratch copy of the sources with -DGC_VPW_MIN_R / _P / _C)
  ab2) V="vr16=variants/vr16/libgcolor.so,vm32=variants/vm32/libgcolor.so,vm32r16=variants/vm32r16/libgcolor.so"
       exec_steps=("abl:rmat24:3:2:base=-,$V" "abl:rmat26:2:1:base=-,$V") ;;
  z3) exec_steps=("profile:uniform10M:--no-cpu-baseline,--no-north-star,--no-variant-b"
                  "profile:mesh512:--no-cpu-baseline,--no-north-star,--no-variant-b") ;;
  # win: one hub per wave with its row window kept across passes (a scratch-copy build, variants/win):
  #    parity with that build, then A/B against the final build
  win) exec_steps=(env:GC_LIB_PATH=variants/win/libgcolor.so "file:tests/test_gpu_hubs.py" "file:tests/test_gpu_parity.py"
                   "file:tests/test_gpu_core.py" "file:tests/test_gpu_fullsize.py:c3_rmat24_against_single_thread_oracle~or~c3_rmat24_hubs_match"
                   env:GC_LIB_PATH= "abl:rmat24:3:2:base=-,win=variants/win/libgcolor.so"
                   "abl:rmat26:2:1:base=-,win=variants/win/libgcolor.so") ;;
  # fin2a / fin2b: the final build (with GC_HUB_WIN) profiled again, its default bench line
  fin2a) exec_steps=(profile:rmat24 "profile:rmat24:--variant,B") ;;
  fin2b) exec_steps=(profile:rmat26 smoke bench:rmat24) ;;
  fin3) exec_steps=(tests smoke) ;;
  fin4) exec_steps=("profile:rmat28:--no-cpu-baseline,--no-north-star,--no-variant-b"
                    "profile:uniform10M:--no-cpu-baseline,--no-north-star,--no-variant-b") ;;
  *) echo "usage: $0 a|..." >&2; exit 2 ;;
esac
bash tools/gpu_session.sh "r06$1" "${exec_steps[@]}"
