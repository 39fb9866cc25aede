#!/bin/bash
# Per-kernel times of the training step (B = 2000) for several library builds:
# one rocprofv3 kernel trace each, the named kernels' average durations.
#   bash tools/gpu_train_kernel_ab.sh TAG 'kernel1|kernel2' lib_a.so lib_b.so ...
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1; PAT=$2; shift 2
mkdir -p gpurun_out; export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename $lib .so)
  HYBRIDFLUX_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ktab_${TAG}_$n -o run -- \
    python3 tools/bench_train.py --batches 2000 --steps 10 --cpu-samples 0 > gpurun_out/ktab_${TAG}_$n.json 2> gpurun_out/ktab_${TAG}_$n.err || exit $?
  db=$(find /tmp/ktab_${TAG}_$n -name "*.db" | head -1)
  python3 tools/rocpd_summary.py "$db" | grep -E "$PAT" | cut -d'|' -f2,3,5 | sed "s/^/$n /"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['gpu']['2000'])" gpurun_out/ktab_${TAG}_$n.json $n
done
