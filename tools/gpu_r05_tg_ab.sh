#!/bin/bash
# Training tests, the training-step kernel trace of the current build, then
# the tgemm A/B (XCD-paired tiles, MFMA-cluster priority) on the training bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tr_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/tr_pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_train_prof.sh r05_fused > gpurun_out/r05_fused_prof.out 2>&1 || exit $?
head -24 gpurun_out/train_kernel_stats_r05_fused.md | cut -c1-200
bash tools/gpu_train_ab.sh tg gnn-plasma-flux_amd/hybridflux/_lib/libhybridflux.so build/ab/lib_xcd.so build/ab/lib_prio.so
