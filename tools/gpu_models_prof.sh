#!/bin/bash
# benchmark_timing.py's methods (tools/bench_models.py) and their rocprofv3
# kernel trace (--kernel-trace --stats only):  bash tools/gpu_models_prof.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-models}
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bench_models.py > gpurun_out/models_$TAG.json 2> gpurun_out/models_$TAG.err || exit 5
cat gpurun_out/models_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_models_$TAG -o run -- python3 tools/bench_models.py --no-cpu --runs 2 \
  > gpurun_out/prof_models_$TAG.log 2>&1 || exit 6
db=$(find gpurun_out/prof_models_$TAG -name "*.db" | head -1)
[ -n "$db" ] && python3 tools/rocpd_summary.py "$db" > gpurun_out/models_kernel_stats_$TAG.md && head -24 gpurun_out/models_kernel_stats_$TAG.md
exit 0
