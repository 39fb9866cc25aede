#!/bin/bash
# Round-4 load-pipelining pass: (1) training GEMM with two-phase stencil loads
# (tgemm.h) and the PINN cross-layer weight pipeline: training + baselines GPU
# tests on the shipped build; (2) the PINN kb-major layout build's baselines
# tests; (3) PINN layout / stagger A/B; (4) training A/B against the previous build.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_baselines.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_pipe_main.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_pipe_main.log; [ $rc -eq 0 ] || exit $rc
HYBRIDFLUX_LIB=build/r04ab/lib_kbmstg.so timeout -k 10 300 python -u -m pytest tests/test_gpu_baselines.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_pipe_kbm.log 2>&1
echo "kbmstg rc=$?"; tail -1 gpurun_out/pytest_pipe_kbm.log
bash tools/gpu_models_ab.sh pinn_layout build/r04ab/lib_a.so build/r04ab/lib_kbm.so build/r04ab/lib_stg.so build/r04ab/lib_kbmstg.so || exit $?
bash tools/gpu_train_ab.sh tg_twophase build/r04ab/lib_head.so build/r04ab/lib_a.so
