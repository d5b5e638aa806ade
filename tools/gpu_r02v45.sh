set -euo pipefail
# sharded engine at N=1 over a one-rank RCCL group (enqueued collectives, no host sync in the
# all-gather): JP sweep seams run ahead of the host (--seam-ahead 4) against one (1)
O=gpurun_out/r02v45; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_shard_gpu.py -x -q --timeout 300 --timeout-method thread > $O/test_shard_gpu.log 2>&1 || { tail -30 $O/test_shard_gpu.log; exit 1; }
tail -2 $O/test_shard_gpu.log
for W in rmat24 mesh256 uniform10M; do
  for A in 1 4; do
    timeout -k 10 300 python -u bench.py --sharded --seam-ahead $A --workload $W --steps 5 --warmup 1 --json-out $O/sh_${W}_a$A.json > $O/sh_${W}_a$A.log 2>&1 || { tail -30 $O/sh_${W}_a$A.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/sh_${W}_a$A.json'));c=d['config'];print('$W a$A',round(d['ms_per_step'],1),c['single_gpu_ms'],c['rounds'],c['exchanges_per_step'],c['sweep_seams_run_ahead'],c['fused_misses'])"
  done
done
