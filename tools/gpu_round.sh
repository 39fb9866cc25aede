#!/bin/bash
# One GPU pass: every GPU test (no -x, measured parity errors recorded), smoke,
# bench; optional extra script after it.  TAG names the outputs.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r02}
EXTRA=${2:-}
mkdir -p gpurun_out; export TMPDIR=/tmp
HF_PARITY_RECORD=gpurun_out/parity_errors_$TAG.json timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
prc=$?
echo "pytest rc=$prc"
tail -1 gpurun_out/pytest_gpu_$TAG.log; grep -E "^FAILED|^ERROR" gpurun_out/pytest_gpu_$TAG.log | head -20
grep -qE "Fatal|core dumped|Aborted|Segmentation" gpurun_out/pytest_gpu_$TAG.log && exit 3
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && cat gpurun_out/smoke_$TAG.log \
 && timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && cat gpurun_out/bench_$TAG.json \
 && { [ -z "$EXTRA" ] || bash $EXTRA $TAG; }
