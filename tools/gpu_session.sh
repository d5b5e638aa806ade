#!/bin/bash
# One gpurun session: a list of steps, each under its own time limit, chained so that the
# first failure ends the session (no GPU step runs after a fault, abort or timeout).
#   bash tools/gpu_session.sh TAG STEP [STEP ...]
# Steps:
#   tests             pytest -m gpu (every GPU test)
#   tests:EXPR        pytest -m gpu -k EXPR (~ stands for a space: not~slow)
#   file:PATH[:EXPR]  pytest -m gpu on one test file (optionally -k EXPR)
#   smoke             __graft_entry__.smoke()
#   bench:WL[:ARGS]   bench.py --workload WL [ARGS, comma-separated]
#   step:WL           tools/step_timing.py WL (phase times of the step)
#   profile:WL[:ARGS] tools/gpu_profile.sh TAG WL [ARGS] (trace + PMC passes, summaries)
#   py:SCRIPT[:ARGS]  python SCRIPT [ARGS, comma-separated] (a tools/ script; 600 s limit)
#   pyl:SCRIPT[:ARGS] the same with an 1100 s limit (fixture builds)
#   env:NAME=VALUE    export NAME=VALUE for the steps after it (env:NAME= unsets it)
#   ubench:NAME[:ARGS] build tools/ubench/NAME.hip for gfx950 and run it (120 s limit)
#   rounds:WL[:SFX]   per-round kernel cost by frontier size (tools/round_cost.py under
#                     rocprofv3 --kernel-trace; the raw trace is deleted after the analysis)
#   brounds:WL        variant B's per-round cost (tools/b_round_cost.py, likewise)
#   torchrun:N[:ARGS] bench.py --gpus N under torch.distributed.run, every rank on GPU 0, gloo
#   ab:WL:REPS:CFGS   tools/ab_steps.py WL REPS CFG... (CFGS comma-separated, each NAME=VAR:val+VAR:val):
#                     interleaved in-process A/B of environment knobs, colourings checked equal
#   abl:WL:REPS:CYCLES:VARS  tools/ab_libs.sh: compile-time variants, a process each, alternated
#                     (VARS comma-separated NAME=PATH, PATH - = the in-tree build)
#   ?STEP             soft step: a plain test failure (pytest rc 1 with no GPU error in its log)
#                     is recorded and the session goes on; anything else still ends it
# Output: gpurun_out/TAG/ (merged back by gpurun).
set -uo pipefail
TAG=$1
shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$TAG
mkdir -p "$O"
cd "$ROOT"
i=0
for st in "$@"; do
  i=$((i + 1))
  soft=0
  if [ "${st:0:1}" = "?" ]; then soft=1; st=${st:1}; fi
  kind=${st%%:*}
  rest=${st#*:}
  [ "$rest" = "$st" ] && rest=""
  rest=${rest//\~/ }
  log="$O/$(printf %02d $i)_${kind}.log"
  echo "== step $i: $st" | tee -a "$O/session.log"
  case $kind in
    tests)
      if [ -n "$rest" ]; then
        timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$rest" > "$log" 2>&1
      else
        timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$log" 2>&1
      fi ;;
    file)
      f=${rest%%:*}; k=${rest#*:}; [ "$k" = "$rest" ] && k=""
      if [ -n "$k" ]; then
        timeout -k 10 1000 python -u -m pytest "$f" -m gpu -x -v --timeout 300 --timeout-method thread -k "$k" > "$log" 2>&1
      else
        timeout -k 10 1000 python -u -m pytest "$f" -m gpu -x -v --timeout 300 --timeout-method thread > "$log" 2>&1
      fi ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1 ;;
    bench)
      wl=${rest%%:*}; a=${rest#*:}; [ "$a" = "$rest" ] && a=""
      timeout -k 10 600 python -u bench.py --workload "$wl" ${a//,/ } --json-out "$O/bench_${wl}.json" > "$log" 2>&1 ;;
    step)
      timeout -k 10 400 python -u tools/step_timing.py "$rest" 4 > "$log" 2>&1 ;;
    profile)
      wl=${rest%%:*}; a=${rest#*:}; [ "$a" = "$rest" ] && a=""
      bash tools/gpu_profile.sh "$TAG" "$wl" ${a//,/ } > "$log" 2>&1 ;;
    env)
      nm=${rest%%=*}; vl=${rest#*=}
      if [ -n "$vl" ]; then export "$nm=$vl"; else unset "$nm"; fi
      true > "$log" ;;
    ubench)
      nm=${rest%%:*}; a=${rest#*:}; [ "$a" = "$rest" ] && a=""
      hipcc --offload-arch=gfx950 -O3 "tools/ubench/$nm.hip" -o "$O/$nm" > "$log" 2>&1 &&
        timeout -k 10 120 "$O/$nm" ${a//,/ } >> "$log" 2>&1 ;;
    calib)
      # FETCH_SIZE / WRITE_SIZE per op of the engine's access patterns (tools/ubench/gather_bytes.hip)
      C=$O/calib
      mkdir -p "$C"
      hipcc --offload-arch=gfx950 -O3 tools/ubench/gather_bytes.hip -o "$C/gather_bytes" > "$log" 2>&1 &&
        timeout -k 10 120 "$C/gather_bytes" 5 > "$C/timing.txt" 2>> "$log" &&
        ( cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d "$C/pmc_fetch" -o run -- "$C/gather_bytes" 5 ) >> "$log" 2>&1 &&
        ( cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d "$C/pmc_write" -o run -- "$C/gather_bytes" 5 ) >> "$log" 2>&1 &&
        python tools/ubench_pmc.py "$C" > "$C/calibration.json" 2>> "$log" && cat "$C/timing.txt" "$C/calibration.json" >> "$log" ;;
    rounds)
      wl=${rest%%:*}; sfx=${rest#*:}; [ "$sfx" = "$rest" ] && sfx=""
      RD="$O/rounds_$wl${sfx:+_$sfx}"
      mkdir -p "$RD"
      ( cd /tmp && TMPDIR=/tmp timeout -k 10 400 rocprofv3 --kernel-trace -T -f csv -d "$RD" -o run -- \
          python3 "$ROOT/tools/round_cost.py" run "$wl" "$RD/records.json" 2 ) > "$log" 2>&1 &&
        tr=$(find "$RD" -name '*kernel_trace.csv' -print -quit) && [ -n "$tr" ] &&
        python tools/round_cost.py analyze "$tr" "$RD/records.json" \
          > "$RD/round_cost.txt" 2>> "$log" &&
        rm -f "$tr" && cat "$RD/round_cost.txt" >> "$log" ;;
    brounds)
      mkdir -p "$O/brounds_$rest"
      ( cd /tmp && TMPDIR=/tmp timeout -k 10 400 rocprofv3 --kernel-trace -T -f csv -d "$O/brounds_$rest" -o run -- \
          python3 "$ROOT/tools/b_round_cost.py" run "$rest" "$O/brounds_$rest/records.json" 2 ) > "$log" 2>&1 &&
        tr=$(find "$O/brounds_$rest" -name '*kernel_trace.csv' -print -quit) && [ -n "$tr" ] &&
        python tools/b_round_cost.py analyze "$tr" "$O/brounds_$rest/records.json" \
          > "$O/brounds_$rest/b_round_cost.txt" 2>> "$log" &&
        rm -f "$tr" && cat "$O/brounds_$rest/b_round_cost.txt" >> "$log" ;;
    torchrun)
      # the N-rank bench on this box's one GPU: every rank pinned to GPU 0 (GC_BENCH_DEVICE),
      # the exchanges over gloo (two processes cannot share a GPU in one RCCL group)
      np_=${rest%%:*}; a=${rest#*:}; [ "$a" = "$rest" ] && a=""
      GC_BENCH_DEVICE=0 GC_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node "$np_" --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus "$np_" ${a//,/ } \
        --json-out "$O/bench_torchrun$np_.json" > "$log" 2>&1 ;;
    py)
      sc=${rest%%:*}; a=${rest#*:}; [ "$a" = "$rest" ] && a=""
      timeout -k 10 600 python -u "$sc" ${a//,/ } > "$log" 2>&1 ;;
    pyl)
      sc=${rest%%:*}; a=${rest#*:}; [ "$a" = "$rest" ] && a=""
      timeout -k 10 1100 python -u "$sc" ${a//,/ } > "$log" 2>&1 ;;
    abl)
      wl=${rest%%:*}; a=${rest#*:}; reps=${a%%:*}; a=${a#*:}; cyc=${a%%:*}; vs=${a#*:}
      timeout -k 10 1100 bash tools/ab_libs.sh "$wl" "$reps" "$cyc" ${vs//,/ } > "$log" 2>&1 &&
        grep "^== " "$log" | grep -v "interleaved" >> "$log.summary"; cat "$log.summary" >> "$log" ;;
    ab)
      wl=${rest%%:*}; a=${rest#*:}; reps=${a%%:*}; cf=${a#*:}
      timeout -k 10 600 python -u tools/ab_steps.py "$wl" "$reps" ${cf//,/ } > "$log" 2>&1 ;;
    *)
      echo "unknown step $st" > "$log"; false ;;
  esac
  rc=$?
  tail -3 "$log" | cut -c1-400 | tee -a "$O/session.log"
  if [ $rc -eq 1 ] && [ $soft -eq 1 ] && ! grep -qE "HSA_STATUS_ERROR|Memory access fault|GPU core dump|hipError|GcolorError|status -2" "$log"; then
    echo "== step $i ($st) FAILED (soft: test failures only, session goes on)" | tee -a "$O/session.log"
    grep -E "^(FAILED|ERROR) " "$log" | head -20 | tee -a "$O/session.log"
    continue
  fi
  if [ $rc -ne 0 ]; then
    echo "== step $i ($st) failed: rc=$rc" | tee -a "$O/session.log"
    tail -40 "$log"
    exit $rc
  fi
done
echo "== session $TAG done" | tee -a "$O/session.log"
