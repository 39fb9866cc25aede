#!/bin/bash
# packed PureGNN + PINN weights in the shipped library: baselines + drop-in GPU tests, then the default bench line
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_baselines.py tests/test_gpu_dropin.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_pack_check.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_pack_check.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_pack_check.json 2> gpurun_out/bench_pack_check.err || exit 5
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_pack_check.json").read())
print(d["value"], d["roofline"]["frac"], d.get("traffic_build"))
for m in d.get("other_models", []):
    print(m.get("model"), m.get("value"), m.get("roofline", {}).get("frac"))
PY
