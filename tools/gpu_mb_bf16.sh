#!/bin/bash
# bf16 layer-loop microbenchmark (tools/microbench/bf16_shape.hip, prebuilt by
# tools/microbench/build.sh): every variant, 6 interleaved rounds.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r04}
mkdir -p gpurun_out
timeout -k 10 120 ./build/mb_bf16_shape 400 > gpurun_out/mb_bf16_$TAG.jsonl 2>&1; rc=$?
tail -8 gpurun_out/mb_bf16_$TAG.jsonl
exit $rc
