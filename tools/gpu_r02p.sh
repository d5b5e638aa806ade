set -euo pipefail
mkdir -p gpurun_out/r02p
STEPS=3 bash tools/gpu_ab.sh r02p mesh512 - "GC_FUSE=0" "GC_SNAP_COPY=1" "GC_FUSE=0 GC_SNAP_COPY=1"
STEPS=3 bash tools/gpu_ab.sh r02p rmat24 - "GC_SNAP_COPY=1"
STEPS=5 bash tools/gpu_ab.sh r02p uniform10M - "GC_FUSE=0" "GC_SNAP_COPY=1"
python - <<'P'
import json,glob
for f in sorted(glob.glob('gpurun_out/r02p/*.json')):
    d=json.load(open(f)); print(f, round(d['ms_per_step'],2), 'event pass', round(d['roofline']['event_pass_ms_per_step'],2))
P
