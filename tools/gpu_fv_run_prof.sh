#!/bin/bash
# rocprofv3 kernel trace + stats of the classical rollout A/B (tools/fv_run_ab.py)
# at nx = 1024 and 512: the one-launch fv_run_fft_kernel beside the per-step
# fv_step_fft_kernel<false> launches (HF_FV_PERSIST=0).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-fvprof}
mkdir -p gpurun_out; export TMPDIR=/tmp
for nx in 1024 512; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$nx -o run -- python3 tools/fv_run_ab.py $nx 4096 30 \
    > gpurun_out/prof_${TAG}_$nx.log 2>&1 || exit 6
  HF_FV_PERSIST=0 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_${nx}_steps -o run -- python3 tools/fv_run_ab.py $nx 4096 30 \
    > gpurun_out/prof_${TAG}_${nx}_steps.log 2>&1 || exit 7
done
find gpurun_out -path "*prof_${TAG}*" -name "*kernel_stats.csv" | sort
