#!/bin/bash
# bf16 layer loop with a scalar trip count (no spilled counter, no vmcnt(0) per
# layer): bf16 precision tests on the shipped build, then the cfg4 A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_precisions.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_bf16fix.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_bf16fix.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_cfg4_ab.sh bf16fix build/r04ab/lib_a.so build/r04ab/lib_b.so
