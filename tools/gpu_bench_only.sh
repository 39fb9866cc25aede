#!/bin/bash
# The default bench and the driver's 20/5 bench of the shipped build (no tests).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-b}
mkdir -p gpurun_out
timeout -k 10 500 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 5
cut -c1-400 gpurun_out/bench_$TAG.json
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_$TAG.json 2> gpurun_out/bench_driver_$TAG.err || exit 6
cut -c1-300 gpurun_out/bench_driver_$TAG.json
