set -euo pipefail
# sharded engine at N=1 over a one-rank RCCL group: inline delta part following the frontiers
# (--seam-inline-max 65536, the default) against the fixed 4096 of before
O=gpurun_out/r02v46; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_shard_gpu.py -x -q --timeout 300 --timeout-method thread > $O/test_shard_gpu.log 2>&1 || { tail -30 $O/test_shard_gpu.log; exit 1; }
tail -2 $O/test_shard_gpu.log
for W in rmat24 mesh256 uniform10M; do
  for M in 4096 65536 4096 65536; do
    timeout -k 10 300 python -u bench.py --sharded --seam-inline-max $M --workload $W --steps 5 --warmup 1 --json-out $O/sh_${W}_m$M.json > $O/sh_${W}_m$M.log 2>&1 || { tail -30 $O/sh_${W}_m$M.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/sh_${W}_m$M.json'));c=d['config'];print('$W m$M',round(d['ms_per_step'],1),c['single_gpu_ms'],c['rounds'],c['exchanges_per_step'],c['sweep_seams_run_ahead'],c['fused_misses'])"
  done
done
