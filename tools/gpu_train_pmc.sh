#!/bin/bash
# PMC passes over the training bench at B = 2000 (tools/bench_train.py): shader
# clock + MFMA busy, instruction mix / waits, HBM bytes; one pass each.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r03}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 tools/bench_train.py --batches 2000 --steps 4 --warmup 2 --cpu-samples 0"
timeout -k 10 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/pmc_tr_$TAG -o p -- $B > gpurun_out/pmc_tr_$TAG.log 2>&1 \
 && timeout -k 10 150 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU --kernel-trace -d gpurun_out/pmc_trsq_$TAG -o p -- $B > gpurun_out/pmc_trsq_$TAG.log 2>&1 \
 && timeout -k 10 150 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --kernel-trace -d gpurun_out/pmc_trhbm_$TAG -o p -- $B > gpurun_out/pmc_trhbm_$TAG.log 2>&1
rc=$?
python3 tools/pmc_summary.py tgemm gpurun_out/pmc_tr_$TAG/*.db gpurun_out/pmc_trsq_$TAG/*.db gpurun_out/pmc_trhbm_$TAG/*.db > gpurun_out/pmc_train_$TAG.txt 2>&1
tail -30 gpurun_out/pmc_train_$TAG.txt
exit $rc
