#!/bin/bash
# Where the FV/FFT step kernel's time goes (fv_step_fft_kernel<false,1024>,
# 4096 ICs, tools/diag_fv.py): SQ counters in two passes (<= 8 SQ each), then
# per-dispatch values and totals (tools/pmc_summary.py).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r03}
mkdir -p gpurun_out
export TMPDIR=/tmp
P="python3 tools/diag_fv.py 1024 4096"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU \
  --kernel-trace -d gpurun_out/pmc_fvs1_$TAG -o p -- $P > gpurun_out/pmc_fvs1_$TAG.log 2>&1 \
 && timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE \
  --kernel-trace -d gpurun_out/pmc_fvs2_$TAG -o p -- $P > gpurun_out/pmc_fvs2_$TAG.log 2>&1
rc=$?
python3 tools/pmc_summary.py "fv_step_fft_kernel<false, 1024>" gpurun_out/pmc_fvs1_$TAG/*.db gpurun_out/pmc_fvs2_$TAG/*.db 2>&1 | tail -8
exit $rc
