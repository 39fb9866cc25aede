#!/bin/bash
# A/B of library builds on BASELINE cfg2 (256 ICs x 64 cells, $PREC (default f32), W1_r1, 50
# steps recording every state): bench.py's headline line per build, alternated twice.
#   bash tools/gpu_ab_cfg2.sh TAG lib_a.so lib_b.so ...
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1
shift
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    HYBRIDFLUX_LIB=$lib timeout -k 10 120 python bench.py --ics-per-gpu 256 --steps 50 --warmup 10 \
      --weights tests/golden/weights_W1_r1.npz --precision ${PREC:-f32} --also= --no-cpu-baseline --no-other-configs \
      > gpurun_out/ab2_${TAG}${PREC:+_$PREC}_${n}_$rep.json 2> gpurun_out/ab2_${TAG}${PREC:+_$PREC}_${n}_$rep.err || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" gpurun_out/ab2_${TAG}${PREC:+_$PREC}_${n}_$rep.json $n $rep
  done
done
