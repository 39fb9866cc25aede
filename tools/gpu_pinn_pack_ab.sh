#!/bin/bash
# PINN one-launch rollout: packed [tile][k-block][lane][4] weights (HF_EXP_PINN_PACK) vs nn.Linear rows;
# parity of the packed build first, then the A/B on tools/bench_models.py
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
HYBRIDFLUX_LIB=build/r04ab/lib_pack.so timeout -k 10 300 python -u -m pytest tests/test_gpu_baselines.py -k "pinn or PINN" -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_pinn_pack.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_pinn_pack.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_models_ab.sh pinn_pack build/r04ab/lib_base.so build/r04ab/lib_pack.so
