#!/bin/bash
# Same-box A/B of the driver's bench command (--steps 20 --warmup 5, headline
# only): the round-1 tree (build/r01_tree, its own library and bench.py) against
# this tree, and this tree with its output buffers first-touched before the
# warmup (HF_BENCH_TOUCH=1).  Three alternating rounds.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r03}
OUT=gpurun_out/core_ab_$TAG.jsonl
: > $OUT
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-other-configs --also="
for i in 1 2 3; do
  (cd build/r01_tree && timeout -k 10 120 python3 bench.py $ARGS) | sed "s/^/{\"arm\": \"r01\", \"i\": $i, \"line\": /; s/\$/}/" >> $OUT || exit 1
  timeout -k 10 120 python3 bench.py $ARGS | sed "s/^/{\"arm\": \"r03\", \"i\": $i, \"line\": /; s/\$/}/" >> $OUT || exit 1
  HF_BENCH_TOUCH=1 timeout -k 10 120 python3 bench.py $ARGS | sed "s/^/{\"arm\": \"r03_touch\", \"i\": $i, \"line\": /; s/\$/}/" >> $OUT || exit 1
  echo "round $i done"
done
python3 - "$OUT" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    d = json.loads(ln); r = d["line"]["roofline"]
    print(d["arm"], d["i"], r["kernel_ms"], r.get("kernel_ms_next_rollout"), r["frac"])
PY
