#!/bin/bash
# A/B of library builds on the training bench (B = 2000), alternated twice:
#   bash tools/gpu_train_ab.sh TAG lib_a.so lib_b.so ...
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1
shift
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    HYBRIDFLUX_LIB=$lib timeout -k 10 200 python3 tools/bench_train.py --batches 2000 --cpu-samples 0 \
      > gpurun_out/trab_${TAG}_${n}_$rep.json 2> gpurun_out/trab_${TAG}_${n}_$rep.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); g=d['gpu']['2000']; print(sys.argv[2], $rep, g['eager_samples_per_s'], g['graphed_samples_per_s'], g['eager_fused_adam_samples_per_s'], d['roofline']['frac'])" gpurun_out/trab_${TAG}_${n}_$rep.json $n
  done
done
