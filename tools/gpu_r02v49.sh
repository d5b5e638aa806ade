set -euo pipefail
# sharded P=1 over a one-rank RCCL group: the process group all-gather with asyncOp False, no propose_block launch on meshes
O=gpurun_out/r02v49; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_shard_gpu.py -x -q --timeout 300 --timeout-method thread > $O/test_shard_gpu.log 2>&1 || { tail -30 $O/test_shard_gpu.log; exit 1; }
tail -2 $O/test_shard_gpu.log
for W in mesh256 rmat24 uniform10M mesh256 rmat24; do
  timeout -k 10 300 python -u bench.py --sharded --workload $W --steps 5 --warmup 1 --json-out $O/sh_$W.json > $O/sh_$W.log 2>&1 || { tail -30 $O/sh_$W.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/sh_$W.json'));c=d['config'];print('$W',round(d['ms_per_step'],1),c['single_gpu_ms'],c['rounds'],c['exchanges_per_step'],c['sweep_seams_run_ahead'],c['fused_misses'])"
done
timeout -k 10 300 python -u tools/shard_cprof.py mesh256 > $O/cprof_mesh256.txt 2>&1 || { tail -30 $O/cprof_mesh256.txt; exit 1; }
grep -E "function calls|all_gather|_allgather|cpu" $O/cprof_mesh256.txt | head -8 | cut -c1-160
