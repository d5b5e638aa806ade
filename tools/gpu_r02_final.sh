set -euo pipefail
# Round-2 evidence: per workload a bench line, rocprofv3 kernel stats and FETCH/WRITE PMC
# passes (tools/gpu_profile.sh); the PMC summaries become profiles/pmc/<workload>.json
# (what bench.py reads for `traffic`), then the default bench line again with them.
T=${1:-r02_final}
for WL in rmat24 mesh512 uniform10M rmat26; do
  bash tools/gpu_profile.sh $T $WL --no-cpu-baseline > gpurun_out/$T.$WL.log 2>&1 || { tail -20 gpurun_out/$T.$WL.log; exit 1; }
  cp gpurun_out/$T/$WL/pmc_summary.json profiles/pmc/$WL.json
  mkdir -p gpurun_out/$T/pmc && cp gpurun_out/$T/$WL/pmc_summary.json gpurun_out/$T/pmc/$WL.json
  echo "$WL profiled"
done
timeout -k 10 600 python -u bench.py --json-out gpurun_out/$T/bench_default.json > gpurun_out/$T/bench_default.log 2>&1 || { tail -20 gpurun_out/$T/bench_default.log; exit 1; }
tail -1 gpurun_out/$T/bench_default.log | cut -c1-400
