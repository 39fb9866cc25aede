#!/bin/bash
# r04 v4: the packed end-of-rollout exchange (Python only; library unchanged):
# distributed + dropin GPU tests, default bench, driver bench
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r04_v4}
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_dropin.py -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; grep -E "^FAILED|^ERROR" gpurun_out/pytest_$TAG.log | head
grep -qE "Fatal|core dumped|Aborted|Segmentation" gpurun_out/pytest_$TAG.log && exit 3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 5
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_$TAG.json 2> gpurun_out/bench_driver_$TAG.err || exit 6
for f in bench bench_driver; do
  python3 -c "import json;d=json.load(open('gpurun_out/${f}_$TAG.json'));r=d['roofline'];print('$f',d['value'],r['frac'],r['kernel_ms'],r['kernel_ms_next_rollout'],r['traffic'],r['traffic_build'],d['config']['collective']['calls'],d['config']['collective']['exchange_ms'],d['parity']['max_err_vs_reference_f32'])"
done
