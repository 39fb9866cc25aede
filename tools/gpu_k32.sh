#!/bin/bash
# K32 cores: precision parity tests, then the bench line with f16x3 alt and cfg4 bf16 (no CPU baseline).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-k}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_precisions.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
cat gpurun_out/bench_$TAG.json
exit $rc
