#!/bin/bash
# A/B of library builds on tools/bench_models.py (no CPU column), alternated twice:
#   bash tools/gpu_models_ab.sh TAG lib_a.so lib_b.so ...
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1
shift
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    HYBRIDFLUX_LIB=$lib timeout -k 10 200 python tools/bench_models.py --no-cpu > gpurun_out/mab_${TAG}_${n}_$rep.json 2> gpurun_out/mab_${TAG}_${n}_$rep.err || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1]))['gpu']; print(sys.argv[2], sys.argv[3], *[(k, v['batched_ic_steps_per_s'], v['single_ic_s'], v.get('frac_of_f32_peak')) for k, v in d.items() if k in ('pinn', 'pure_gnn')])" gpurun_out/mab_${TAG}_${n}_$rep.json $n $rep
  done
done
