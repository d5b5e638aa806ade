set -euo pipefail
# layout probe: mesh in natural vs diagonal-band numbering
T=r02v4; mkdir -p gpurun_out/$T
timeout -k 10 300 python -u tools/relabel_probe.py 256 > gpurun_out/$T/probe256.log 2>&1; cat gpurun_out/$T/probe256.log
timeout -k 10 500 python -u tools/relabel_probe.py 512 > gpurun_out/$T/probe512.log 2>&1; cat gpurun_out/$T/probe512.log
