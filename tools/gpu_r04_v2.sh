#!/bin/bash
# r04 v2: distributed / lanes / bf16 tests, cfg4 lane-cut A/B, driver bench x2
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_precisions.py -k "distributed or layers_and_nx or lanes or cfg4" -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r04_v2.log 2>&1
rc=$?; tail -16 gpurun_out/pytest_r04_v2.log
grep -qE "Fatal|core dumped|Aborted|Segmentation" gpurun_out/pytest_r04_v2.log && exit 3
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  HF_LANE_CUTS=even timeout -k 10 120 python3 tools/cfg4_lanes_ab.py even$i >> gpurun_out/cfg4_lanes_ab_r04_v2.jsonl || exit 5
  timeout -k 10 120 python3 tools/cfg4_lanes_ab.py rounds$i >> gpurun_out/cfg4_lanes_ab_r04_v2.jsonl || exit 6
done
cat gpurun_out/cfg4_lanes_ab_r04_v2.jsonl
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-other-configs --also= > gpurun_out/bench_driver_r04_v2_$i.json 2>/dev/null || exit 7
  python3 -c "import json;d=json.load(open('gpurun_out/bench_driver_r04_v2_$i.json'));print(d['value'],d['roofline']['kernel_ms'],d['roofline']['kernel_ms_next_rollout'],d['config']['collective']['exchange_ms'])"
done
