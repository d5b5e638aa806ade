set -euo pipefail
bash tools/gpu_profile.sh r02w uniform10M > /dev/null
bash tools/gpu_profile.sh r02wB rmat24 --variant B > /dev/null
bash tools/gpu_profile.sh r02wB uniform10M --variant B > /dev/null
for w in r02w/uniform10M r02wB/rmat24 r02wB/uniform10M; do tail -1 gpurun_out/$w/bench.log | cut -c1-250; done
