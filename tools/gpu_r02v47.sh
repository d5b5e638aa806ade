set -euo pipefail
# host profile of one P=1 sharded colouring over a one-rank RCCL group
O=gpurun_out/r02v47; mkdir -p $O
for W in mesh256 rmat24; do
  timeout -k 10 300 python -u tools/shard_cprof.py $W > $O/cprof_$W.txt 2>&1 || { tail -30 $O/cprof_$W.txt; exit 1; }
  head -45 $O/cprof_$W.txt | cut -c1-150
done
