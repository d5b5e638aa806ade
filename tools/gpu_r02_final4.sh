set -euo pipefail
# final evidence for the default workload (R-MAT-24) and the mesh on the final build
T=r02_final4
for WL in rmat24 mesh512; do
  bash tools/gpu_profile.sh $T $WL --no-cpu-baseline > gpurun_out/$T.$WL.log 2>&1 || { tail -20 gpurun_out/$T.$WL.log; exit 1; }
  cp gpurun_out/$T/$WL/pmc_summary.json profiles/pmc/$WL.json
  mkdir -p gpurun_out/$T/pmc && cp gpurun_out/$T/$WL/pmc_summary.json gpurun_out/$T/pmc/$WL.json
  echo "$WL profiled"
done
timeout -k 10 600 python -u bench.py --json-out gpurun_out/$T/bench_default.json > gpurun_out/$T/bench_default.log 2>&1 || { tail -20 gpurun_out/$T/bench_default.log; exit 1; }
tail -1 gpurun_out/$T/bench_default.log | cut -c1-300
