#!/bin/bash
# The one A/B driver of library builds on one GPU box (each arm alternated
# twice, HYBRIDFLUX_LIB selects the build; outputs gpurun_out/ab_<MODE>_<TAG>_*):
#   bash tools/gpu_ab.sh MODE TAG lib_a.so lib_b.so ...
# MODE:
#   bench   bench.py's headline line (no CPU baseline / other configs / alt;
#           BENCH_ARGS adds flags)
#   cfg2    BASELINE cfg2 (256 ICs x 64, $PREC or f32, W1_r1, 50 steps)
#   cfg4    BASELINE cfg4 (4096 ICs x 1024, bf16, W1_r2, 30 steps, no trajectory)
#   cfg4tl  tools/cfg4_timeline.py run (cfg4 + random-weight L = 0 / 4 rollouts)
#   diag4   tools/diag_cfg4.py 10 (per-layer slope on the cfg4 grid)
#   train   tools/bench_train.py at B = 2000 (CONFIG=physics|full|...)
#   trainks rocprofv3 kernel trace of the B = 2000 training step, the kernels
#           matching $PAT
#   models  tools/bench_models.py (PureGNN / PINN, no CPU column)
# TESTS=1 first runs tests/test_gpu_training.py (train modes) and stops on a failure.
# (Replaces the per-round one-offs gpu_ab_cfg2.sh, gpu_ab_cfg4.sh,
# gpu_train_ab.sh, gpu_train_kernel_ab.sh, gpu_models_ab.sh, gpu_diag_cfg4.sh and
# gpu_r05_*.sh that earlier profiles name: same commands, same outputs.)
set -o pipefail
cd "$(dirname "$0")/.."
MODE=$1; TAG=$2; shift 2
mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/ab_tests_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/ab_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
show() {  # the arm's figures from its JSON output
  python3 - "$@" <<'PY'
import json, sys
mode, path, n, rep = sys.argv[1:5]
d = json.load(open(path))
if mode in ("bench", "cfg2", "cfg4"):
    print(n, rep, d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])
elif mode == "cfg4tl":
    print(n, rep, [(g["name"], round(g["ms_per_step"], 4)) for g in d["groups"]])
elif mode == "diag4":
    print(n, rep, json.dumps(d))
elif mode in ("train", "trainks"):
    g = d["gpu"]["2000"]
    print(n, rep, g["eager_samples_per_s"], g["graphed_samples_per_s"], g.get("eager_flat_adam_samples_per_s"), g["graphed_flat_adam_samples_per_s"],
          d["roofline"]["frac"])
elif mode == "models":
    g = d["gpu"]
    print(n, rep, *[(k, v["batched_ic_steps_per_s"], v.get("frac_of_f32_peak")) for k, v in g.items()
                    if k in ("pinn", "pure_gnn")])
PY
}
reps="1 2"; [ "$MODE" = trainks ] && reps=1
for rep in $reps; do
  for lib in "$@"; do
    n=$(basename $lib .so); o=gpurun_out/ab_${MODE}_${TAG}_${n}_$rep
    export HYBRIDFLUX_LIB=$lib
    case $MODE in
      bench) timeout -k 10 150 python bench.py --no-cpu-baseline --no-other-configs --also= $BENCH_ARGS ;;
      cfg2) timeout -k 10 120 python bench.py --ics-per-gpu 256 --steps 50 --warmup 10 \
              --weights tests/golden/weights_W1_r1.npz --precision ${PREC:-f32} --also= --no-cpu-baseline --no-other-configs ;;
      cfg4) timeout -k 10 120 python bench.py --nx 1024 --precision bf16 --ics-per-gpu 4096 --steps 30 --warmup 3 \
              --weights tests/golden/weights_W1_r2.npz --no-traj --also= --no-cpu-baseline --no-other-configs ;;
      cfg4tl) timeout -k 10 120 python3 tools/cfg4_timeline.py run ;;
      diag4) timeout -k 10 120 python3 tools/diag_cfg4.py 10 ;;
      train) timeout -k 10 200 python3 tools/bench_train.py --config ${CONFIG:-physics} --batches 2000 --cpu-samples 0 ;;
      trainks) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ab_trainks_${TAG}_$n -o run -- \
                 python3 tools/bench_train.py --config ${CONFIG:-physics} --batches 2000 --steps 10 --cpu-samples 0 ;;
      models) timeout -k 10 200 python tools/bench_models.py --no-cpu ;;
      *) echo "unknown MODE $MODE"; exit 2 ;;
    esac > $o.json 2> $o.err || exit $?
    show $MODE $o.json $n $rep
    if [ $MODE = trainks ]; then
      db=$(find /tmp/ab_trainks_${TAG}_$n -name "*.db" | head -1)
      python3 tools/rocpd_summary.py "$db" > $o.md && grep -E "${PAT:-kernel}" $o.md | cut -d'|' -f2,3,5 | sed "s/^/$n /"
      python3 tools/train_timeline.py "$db" > $o.timeline.md || exit 9
    fi
  done
done
