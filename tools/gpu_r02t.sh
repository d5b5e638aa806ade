set -euo pipefail
bash tools/gpu_pmc_sq.sh r02t_mesh --workload mesh512 --no-event-timing
python tools/pmc_kernels.py gpurun_out/r02t_mesh/sq/run_counter_collection.csv k_commit k_resolve
python tools/pmc_kernels.py gpurun_out/r02t_mesh/tcc/run_counter_collection.csv k_commit k_resolve
