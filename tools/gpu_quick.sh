#!/bin/bash
# quick: parity tests (f32 chain) + bench headline only
set -o pipefail
cd /root/repo
TAG=${1:-q}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_precisions.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline --no-other-configs > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
cat gpurun_out/bench_$TAG.json
exit $rc
