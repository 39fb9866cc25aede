#!/bin/bash
# After gpu_round.sh's bench: the driver's 20/5 command, the plain 2-rank
# self-launch (gloo, both ranks on the one GPU) and the bench's kernel traces.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r03}
bash tools/gpu_driver_bench.sh $TAG || exit 1
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-other-configs --no-cpu-baseline --also= \
  > gpurun_out/bench_gloo2_$TAG.json 2> gpurun_out/bench_gloo2_$TAG.err && cat gpurun_out/bench_gloo2_$TAG.json || exit 2
bash tools/gpu_bench_prof.sh $TAG
