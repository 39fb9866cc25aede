#!/bin/bash
# Timing-diagnostic pass: tools/diag_rollout.py against the real library and each
# diag build (tools/build_diag.sh); one JSON line per library.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-d}
shift
mkdir -p gpurun_out
timeout -k 10 120 python tools/diag_rollout.py > gpurun_out/diag_${TAG}_base.json || exit $?
for v in "$@"; do
  HYBRIDFLUX_LIB=build/diag/lib_$v.so timeout -k 10 120 python tools/diag_rollout.py > gpurun_out/diag_${TAG}_$v.json || exit $?
done
head -50 gpurun_out/diag_${TAG}_*.json
