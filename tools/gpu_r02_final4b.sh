set -euo pipefail
# final evidence, part 2: the north-star scale (R-MAT-26), C2, variant B and smoke() on the final build
T=r02_final4
for WL in rmat26 uniform10M; do
  bash tools/gpu_profile.sh $T $WL --no-cpu-baseline > gpurun_out/$T.$WL.log 2>&1 || { tail -20 gpurun_out/$T.$WL.log; exit 1; }
  mkdir -p gpurun_out/$T/pmc && cp gpurun_out/$T/$WL/pmc_summary.json gpurun_out/$T/pmc/$WL.json
  echo "$WL profiled"
done
timeout -k 10 400 python -u bench.py --variant B --no-cpu-baseline --json-out gpurun_out/$T/bench_rmat24_B.json > gpurun_out/$T/bench_rmat24_B.log 2>&1 || { tail -20 gpurun_out/$T/bench_rmat24_B.log; exit 1; }
tail -1 gpurun_out/$T/bench_rmat24_B.log | cut -c1-300
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
