#!/bin/bash
# HBM traffic of cfg4's FV/FFT kernel (fv_step_fft_kernel<true,1024>) from
# rocprofv3 PMC: FETCH_SIZE and WRITE_SIZE in separate passes (TCC counter
# limits), then per-dispatch values (tools/pmc_summary.py).  FETCH_SIZE is in
# KiB and needs the gfx950 x2 wide-load correction (MI355X_MICROARCH.md).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r02}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --nx 1024 --precision bf16 --steps 5 --warmup 1 --weights tests/golden/weights_W1_r2.npz --no-traj --also= --no-cpu-baseline --no-other-configs"
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fvf_$TAG -o p -- $B > gpurun_out/pmc_fvf_$TAG.log 2>&1 \
 && timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_fvw_$TAG -o p -- $B > gpurun_out/pmc_fvw_$TAG.log 2>&1
rc=$?
python3 tools/pmc_summary.py fv_step_fft gpurun_out/pmc_fvf_$TAG/*.db gpurun_out/pmc_fvw_$TAG/*.db 2>&1 | tail -12
exit $rc
