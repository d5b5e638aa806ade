set -euo pipefail
mkdir -p gpurun_out/hubT
timeout -k 10 600 python -u -m pytest tests/test_gpu_hubs.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hubT/pytest.log 2>&1 || { tail -60 gpurun_out/hubT/pytest.log; exit 1; }
tail -2 gpurun_out/hubT/pytest.log
for t in ${TS:-64 256 1024}; do
  GC_HUB_T=$t timeout -k 10 200 python -u bench.py --workload ${WL:-rmat24} --steps 2 --warmup 1 --no-cpu-baseline --json-out gpurun_out/hubT/bench_$t.json > gpurun_out/hubT/bench_$t.log 2>&1
  python -c "
import json;d=json.load(open('gpurun_out/hubT/bench_$t.json'))
print('$t', round(d['ms_per_step'],1), d['config']['jp_extra_sweeps'], {k:(round(v['ms'],1),v['launches']) for k,v in d.get('kernels_probe_step').items()})"
done
