#!/bin/bash
# cfg4 (4096 x 1024, bf16, T = 30) A/B of library builds, alternated three times
# (tools/cfg4_lanes_ab.py: 0.3 s warm-up, 3 timed rollouts each):
#   bash tools/gpu_cfg4_ab.sh TAG lib_a.so lib_b.so ...
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1
shift
mkdir -p gpurun_out
for rep in 1 2 3; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    HYBRIDFLUX_LIB=$lib timeout -k 10 200 python tools/cfg4_lanes_ab.py ${n}_$rep >> gpurun_out/c4ab_$TAG.jsonl 2> gpurun_out/c4ab_${TAG}_${n}_$rep.err || exit $?
    tail -1 gpurun_out/c4ab_$TAG.jsonl | cut -c1-200
  done
done
