set -euo pipefail
bash tools/gpu_profile.sh r02u rmat26 > /dev/null
bash tools/gpu_profile.sh r02u mesh512 > /dev/null
for w in rmat26 mesh512; do tail -1 gpurun_out/r02u/$w/bench.log | cut -c1-300; done
