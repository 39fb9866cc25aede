#!/bin/bash
# Training tests and the training-step kernel trace of the current build.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-r05_b}
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tr_pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/tr_pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_train_prof.sh $TAG > gpurun_out/prof_$TAG.out 2>&1 || exit $?
head -16 gpurun_out/train_kernel_stats_$TAG.md | cut -c1-160
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps(d['gpu']['2000']), d['roofline']['frac'])" gpurun_out/train_bench_$TAG.json
[ -f build/ab/lib_pipe.so ] && bash tools/gpu_train_ab.sh pipe gnn-plasma-flux_amd/hybridflux/_lib/libhybridflux.so build/ab/lib_pipe.so
exit 0
