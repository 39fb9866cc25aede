#!/bin/bash
# cfg4 lane timeline and fixed-part attribution:
# rocprofv3 kernel trace of tools/cfg4_timeline.py run (shipped library), its
# analysis, then the same run without the profiler for the shipped library and
# every timing-only build under build/d5 (HF_DIAG_*: wrong results by
# construction), alternated twice.   bash tools/gpu_cfg4_timeline.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r06}
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/tl_$TAG -o run -- python3 tools/cfg4_timeline.py run \
  > gpurun_out/tl_run_$TAG.json 2> gpurun_out/tl_run_$TAG.err || exit 7
db=$(find /tmp/tl_$TAG -name "*.db" | head -1)
python3 tools/cfg4_timeline.py analyze "$db" > gpurun_out/tl_analysis_$TAG.json || exit 8
python3 -c "import json;d=json.load(open('gpurun_out/tl_analysis_$TAG.json'));[print({k:v for k,v in r.items() if k not in ('first_rollout_dispatches_us',)}) for r in d['rows']]"
for rep in 1 2; do
  for lib in gnn-plasma-flux_amd/hybridflux/_lib/libhybridflux.so build/d5/lib_*.so; do
    n=$(basename $lib .so)
    HYBRIDFLUX_LIB=$lib timeout -k 10 120 python3 tools/cfg4_timeline.py run > gpurun_out/tl_${TAG}_${n}_$rep.json 2> gpurun_out/tl_${TAG}_${n}_$rep.err || exit 9
    echo "$n $rep $(python3 -c "import json;d=json.load(open('gpurun_out/tl_${TAG}_${n}_$rep.json'));print([(g['name'],round(g['ms_per_step'],4)) for g in d['groups']])")"
  done
done
