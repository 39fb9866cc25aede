#!/bin/bash
# bf16 core: precision parity tests, cfg4 bench line (other_configs), bf16 layer diagnostics.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-bf}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_precisions.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python bench.py --no-cpu-baseline --also '' > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
cat gpurun_out/bench_$TAG.json
DIAG_PREC=bf16 timeout -k 10 120 python tools/diag_rollout.py > gpurun_out/diag_${TAG}_bf16.json
rc=$?
cat gpurun_out/diag_${TAG}_bf16.json
exit $rc
