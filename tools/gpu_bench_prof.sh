#!/bin/bash
# rocprofv3 kernel trace (--kernel-trace --stats only) of the default bench
# command and of the driver's --steps 20 --warmup 5 command, summarised per
# kernel:  bash tools/gpu_bench_prof.sh TAG  (databases under /tmp on the box:
# gpurun copies back at most 64 MiB of gpurun_out/)
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r03}
mkdir -p gpurun_out; export TMPDIR=/tmp
for arm in default driver; do
  args=""; [ $arm = driver ] && args="--gpus 1 --steps 20 --warmup 5"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_bench_${arm}_$TAG -o bench -- python3 bench.py $args \
    > gpurun_out/prof_bench_${arm}_$TAG.json 2> gpurun_out/prof_bench_${arm}_$TAG.err || exit 7
  tail -1 gpurun_out/prof_bench_${arm}_$TAG.json | cut -c1-300
  db=$(find /tmp/prof_bench_${arm}_$TAG -name "*.db" | head -1)
  [ -n "$db" ] && python3 tools/rocpd_summary.py "$db" > gpurun_out/bench_kernel_stats_${arm}_$TAG.md && head -8 gpurun_out/bench_kernel_stats_${arm}_$TAG.md
done
exit 0
