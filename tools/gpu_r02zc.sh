set -euo pipefail
bash tools/gpu_profile.sh r02zc rmat24 > /dev/null
bash tools/gpu_profile.sh r02zc mesh512 > /dev/null
for w in rmat24 mesh512; do tail -1 gpurun_out/r02zc/$w/bench.log | cut -c1-200; done
