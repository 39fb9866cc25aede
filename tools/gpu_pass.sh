#!/bin/bash
# One GPU pass of the shipped build: every GPU test (parity errors recorded),
# smoke, the default bench and the driver's 20/5 bench.  TAG names the
# outputs under gpurun_out/.  Each GPU step has its own time limit; the pass
# stops at the first step that faults, aborts or times out.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-pass}
mkdir -p gpurun_out; export TMPDIR=/tmp
HF_PARITY_RECORD=gpurun_out/parity_errors_$TAG.json timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
prc=$?
echo "pytest rc=$prc"; tail -1 gpurun_out/pytest_gpu_$TAG.log; grep -E "^FAILED|^ERROR" gpurun_out/pytest_gpu_$TAG.log | head -30
case $prc in 124|134|137|139) exit 3;; esac
grep -qE "Fatal|core dumped|Aborted|Segmentation|Memory access fault" gpurun_out/pytest_gpu_$TAG.log && exit 3
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && cat gpurun_out/smoke_$TAG.log || exit 4
timeout -k 10 500 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 5
cut -c1-600 gpurun_out/bench_$TAG.json
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_$TAG.json 2> gpurun_out/bench_driver_$TAG.err || exit 6
cut -c1-300 gpurun_out/bench_driver_$TAG.json
exit $prc
