#!/bin/bash
# f32 tanh_fast in the PureGNN / PINN one-launch rollouts vs device-libm tanhf:
# baselines + drop-in tests on the tanh_fast build, then the A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
HF_PARITY_RECORD=gpurun_out/parity_errors_tanh.json HYBRIDFLUX_LIB=build/r04ab/lib_tf.so timeout -k 10 300 python -u -m pytest tests/test_gpu_baselines.py tests/test_gpu_dropin.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_tanh.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_tanh.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_models_ab.sh tanh build/r04ab/lib_head.so build/r04ab/lib_tf.so
