set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
HF_PARITY_RECORD=gpurun_out/parity_errors_r02_v1.json timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_r02_v1.log 2>&1
echo "pytest rc=$?"
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r02_v1.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_r02_v1.json 2> gpurun_out/bench_r02_v1.err && \
bash tools/gpu_pmc2.sh r02_v1 > gpurun_out/pmc2_r02_v1.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu_r02_v1.log; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu_r02_v1.log | head -20
cat gpurun_out/smoke_r02_v1.log gpurun_out/bench_r02_v1.json; tail -3 gpurun_out/bench_r02_v1.err
exit $rc
