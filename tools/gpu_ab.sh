#!/bin/bash
# A/B of library builds on one box: headline bench (no CPU baseline, no other
# configs, no alt) for each library, alternated twice.  Usage:
#   [BENCH_ARGS="--nx 1024 --precision bf16 --steps 10 --warmup 2"] bash tools/gpu_ab.sh TAG lib_a.so lib_b.so ...
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1
shift
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    HYBRIDFLUX_LIB=$lib timeout -k 10 150 python bench.py --no-cpu-baseline --no-other-configs --also= $BENCH_ARGS > gpurun_out/ab_${TAG}_${n}_$rep.json 2> gpurun_out/ab_${TAG}_${n}_$rep.err || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['roofline']['kernel_ms'], (d.get('alt') or {}).get('f16x3', {}).get('kernel_ms'))" gpurun_out/ab_${TAG}_${n}_$rep.json $n $rep
  done
done
