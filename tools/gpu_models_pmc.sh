#!/bin/bash
# PMC passes over the PureGNN / PINN one-launch rollouts (tools/bench_models.py,
# 4096 ICs x 64 cells, 50 steps): clock + MFMA busy, instruction mix / waits,
# L2 hits; one counter set per run.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r04}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 tools/bench_models.py --no-cpu --runs 2"
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/pmc_m1_$TAG -o p -- $B > gpurun_out/pmc_m1_$TAG.log 2>&1 \
 && timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU --kernel-trace -d gpurun_out/pmc_m2_$TAG -o p -- $B > gpurun_out/pmc_m2_$TAG.log 2>&1 \
 && timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d gpurun_out/pmc_m3_$TAG -o p -- $B > gpurun_out/pmc_m3_$TAG.log 2>&1
rc=$?
for k in pinn_run_kernel pure_run_kernel; do
  python3 tools/pmc_summary.py $k gpurun_out/pmc_m[123]_$TAG/*.db 2>&1 | grep TOTAL
done > gpurun_out/pmc_models_$TAG.txt
cat gpurun_out/pmc_models_$TAG.txt
exit $rc
