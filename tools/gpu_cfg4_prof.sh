#!/bin/bash
# Kernel trace of the nx=1024 (config 4) path and of config 2.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg4_$TAG -o p -- python3 bench.py --nx 1024 --precision bf16 --steps 10 --warmup 2 --also "" --no-cpu-baseline > gpurun_out/prof_cfg4_$TAG.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg2_$TAG -o p -- python3 bench.py --ics-per-gpu 256 --also "" --no-cpu-baseline > gpurun_out/prof_cfg2_$TAG.log 2>&1
