#!/bin/bash
# PINN / PureGNN one-launch rollouts with the weight stream pinned as a software
# pipeline (scheduling barriers per k-block; HF_PINN_AHEAD = k-blocks in flight;
# "x" builds carry it across layers and steps, "nx" builds restart it per layer):
# baselines tests on the shipped build, then the A/B against the earlier builds
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-pinn_pipe}
shift
timeout -k 10 300 python -u -m pytest tests/test_gpu_baselines.py tests/test_gpu_dropin.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_models_ab.sh $TAG "$@"
