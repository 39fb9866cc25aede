#!/bin/bash
# cfg4 (nx=1024, bf16, W1_r2) PMC passes for the windowed flux kernel: shader
# clock + MFMA busy, then instruction mix / waits, one pass each.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r02}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --nx 1024 --precision bf16 --steps 5 --warmup 1 --weights tests/golden/weights_W1_r2.npz --no-traj --also= --no-cpu-baseline --no-other-configs"
timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/pmc_c4_$TAG -o p -- $B > gpurun_out/pmc_c4_$TAG.log 2>&1 \
 && timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU --kernel-trace -d gpurun_out/pmc_c4sq_$TAG -o p -- $B > gpurun_out/pmc_c4sq_$TAG.log 2>&1
rc=$?
python3 tools/pmc_summary.py chain_flux gpurun_out/pmc_c4_$TAG/*.db gpurun_out/pmc_c4sq_$TAG/*.db > gpurun_out/pmc_cfg4_$TAG.txt 2>&1; grep TOTAL gpurun_out/pmc_cfg4_$TAG.txt
exit $rc
