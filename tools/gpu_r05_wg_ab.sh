#!/bin/bash
# Training tests on the shipped build, its training-step kernel trace, then
# the A/B against every build/ab/lib_*.so (AB_TAG names the outputs).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-r05_wg}
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tr_pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/tr_pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_train_prof.sh $TAG > gpurun_out/prof_$TAG.out 2>&1 || exit $?
head -14 gpurun_out/train_kernel_stats_$TAG.md | cut -c1-160
bash tools/gpu_train_ab.sh ${AB_TAG:-ab} gnn-plasma-flux_amd/hybridflux/_lib/libhybridflux.so build/ab/lib_*.so
