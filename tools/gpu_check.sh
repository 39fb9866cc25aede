#!/bin/bash
# One GPU-box pass: parity tests -> smoke -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
HF_PARITY_RECORD=gpurun_out/parity_errors_$TAG.json timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1 \
 && timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
 && timeout -k 10 240 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
 && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o bench -- python3 bench.py --no-cpu-baseline --no-other-configs > gpurun_out/prof_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu_$TAG.log
cat gpurun_out/bench_$TAG.json 2>/dev/null
exit $rc
