#!/bin/bash
# PMC passes over one precision's rollout kernel: MFMA busy, wait states, LDS.
#   bash tools/gpu_pmc_core.sh TAG PRECISION ["extra bench args"] [kernel-name substring]
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r01}
PREC=${2:-f32}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --also= --precision $PREC ${3:-}"
K=${4:-chain_rollout}
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/pmcA_$TAG -o p -- $B > gpurun_out/pmcA_$TAG.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU --kernel-trace -d gpurun_out/pmcB_$TAG -o p -- $B > gpurun_out/pmcB_$TAG.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace -d gpurun_out/pmcC_$TAG -o p -- $B > gpurun_out/pmcC_$TAG.log 2>&1
rc=$?
python3 tools/pmc_summary.py $K $(ls gpurun_out/pmc[ABC]_$TAG/*.db 2>/dev/null) || true
exit $rc
