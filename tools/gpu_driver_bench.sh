#!/bin/bash
# The driver's own bench command (BENCH_rNN.json: --steps 20 --warmup 5), run
# after gpu_round.sh's default bench:  bash tools/gpu_driver_bench.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r03}
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_$TAG.json 2> gpurun_out/bench_driver_$TAG.err \
  && cat gpurun_out/bench_driver_$TAG.json
