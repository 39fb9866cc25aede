set -o pipefail
cd /root/repo
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tr_pytest_pl.log 2>&1; rc=$?; tail -1 gpurun_out/tr_pytest_pl.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for arm in new old; do
    if [ $arm = old ]; then export HF_AB_PLAIN_BATCH=1 HF_AB_NO_FLAT=1; else unset HF_AB_PLAIN_BATCH HF_AB_NO_FLAT; fi
    timeout -k 10 200 python3 tools/bench_train.py --batches 2000 --cpu-samples 0 > gpurun_out/trab_pl_${arm}_$rep.json 2> gpurun_out/trab_pl_${arm}_$rep.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); g=d['gpu']['2000']; print(sys.argv[2], $rep, g['eager_samples_per_s'], g['graphed_samples_per_s'], g['eager_fused_adam_samples_per_s'], d['roofline']['frac'])" gpurun_out/trab_pl_${arm}_$rep.json $arm
  done
done
