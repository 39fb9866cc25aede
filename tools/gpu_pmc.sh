#!/bin/bash
# PMC passes for the roofline's `traffic` and MFMA-utilisation evidence.
# Each counter group is its own rocprofv3 run (kernel trace only, no sys/runtime trace).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r01}
STEPS=${2:-50}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc_list_$TAG.txt 2>&1
B="python3 bench.py --no-cpu-baseline --no-other-configs --also= --steps $STEPS"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_$TAG -o p -- $B > gpurun_out/pmc_fetch_$TAG.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_$TAG -o p -- $B > gpurun_out/pmc_write_$TAG.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc_mfma_$TAG -o p -- $B > gpurun_out/pmc_mfma_$TAG.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace -d gpurun_out/pmc_sq_$TAG -o p -- $B > gpurun_out/pmc_sq_$TAG.log 2>&1
rc=$?
ls gpurun_out/
exit $rc
