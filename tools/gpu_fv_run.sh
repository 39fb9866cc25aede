#!/bin/bash
# Persistent classical rollout at FFT sizes: its parity tests, then the A/B of
# one launch vs per-step launches (tools/fv_run_ab.py) at nx = 256, 512, 1024.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-fvrun}
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "classical or poisson or dataset or compare or large_nx or aliased or generate" > gpurun_out/pytest_$TAG.log 2>&1
prc=$?; tail -3 gpurun_out/pytest_$TAG.log; grep -E "^FAILED|^ERROR" gpurun_out/pytest_$TAG.log | head
[ $prc -eq 0 ] || exit $prc
: > gpurun_out/ab_$TAG.jsonl
for nx in 1024 512 256 64; do
  for p in 0 1; do
    HF_FV_PERSIST=$p timeout -k 10 120 python tools/fv_run_ab.py $nx 4096 30 >> gpurun_out/ab_$TAG.jsonl || exit 5
  done
done
cat gpurun_out/ab_$TAG.jsonl
