#!/bin/bash
# L2 passes over the PureGNN / PINN one-launch rollouts (tools/models_once.py:
# bench.py's other_models workload): L1 -> L2 read requests and their latency,
# L2 hits / misses / requests, then the MFMA-busy and wait counters.  One
# counter set per run; the summary names each dispatch's counts.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r05}
mkdir -p gpurun_out
export TMPDIR=/tmp
P="python3 tools/models_once.py"
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace -d gpurun_out/pmc_l2a_$TAG -o p -- $P > gpurun_out/pmc_l2a_$TAG.log 2>&1 \
 && timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/pmc_l2b_$TAG -o p -- $P > gpurun_out/pmc_l2b_$TAG.log 2>&1 \
 && timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD --kernel-trace -d gpurun_out/pmc_l2c_$TAG -o p -- $P > gpurun_out/pmc_l2c_$TAG.log 2>&1
rc=$?
for k in pinn_run_kernel pure_run_kernel; do
  echo "== $k"
  python3 tools/pmc_summary.py $k gpurun_out/pmc_l2[abc]_$TAG/*.db 2>&1
done > gpurun_out/pmc_models_l2_$TAG.txt
cat gpurun_out/pmc_models_l2_$TAG.txt
exit $rc
