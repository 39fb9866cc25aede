#!/bin/bash
# cfg2 (256 ICs x 64 cells, f32, cell-split kernel) PMC passes: shader clock +
# MFMA busy, then instruction mix / waits, one pass each (tools/pmc_summary.py).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r02}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --ics-per-gpu 256 --steps 50 --warmup 5 --weights tests/golden/weights_W1_r1.npz --also= --no-cpu-baseline --no-other-configs"
timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/pmc_c2_$TAG -o p -- $B > gpurun_out/pmc_c2_$TAG.log 2>&1 \
 && timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU --kernel-trace -d gpurun_out/pmc_c2sq_$TAG -o p -- $B > gpurun_out/pmc_c2sq_$TAG.log 2>&1
rc=$?
python3 tools/pmc_summary.py cells_kernel gpurun_out/pmc_c2_$TAG/*.db gpurun_out/pmc_c2sq_$TAG/*.db 2>&1 | tail -12
exit $rc
