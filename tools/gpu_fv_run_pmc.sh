#!/bin/bash
# HBM traffic of the one-launch classical rollout (fv_run_fft_kernel<1024>) from
# rocprofv3 PMC, FETCH_SIZE and WRITE_SIZE in separate passes; per-dispatch
# values via tools/pmc_summary.py (FETCH_SIZE KiB, x2 gfx950 wide-load
# correction, MI355X_MICROARCH.md).  Workload: tools/fv_run_ab.py 1024 4096 30
# (6 rollouts with trajectory + metrics, 7 final-only).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r02}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fvrf_$TAG -o p -- python3 tools/fv_run_ab.py 1024 4096 30 > gpurun_out/pmc_fvrf_$TAG.log 2>&1 \
 && timeout -k 10 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_fvrw_$TAG -o p -- python3 tools/fv_run_ab.py 1024 4096 30 > gpurun_out/pmc_fvrw_$TAG.log 2>&1
rc=$?
python3 tools/pmc_summary.py fv_run_fft gpurun_out/pmc_fvrf_$TAG/*.db gpurun_out/pmc_fvrw_$TAG/*.db 2>&1 | tail -20
exit $rc
