set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tr_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/tr_pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_train_ab.sh fused gnn-plasma-flux_amd/hybridflux/_lib/libhybridflux.so build/ab/lib_unfused.so
