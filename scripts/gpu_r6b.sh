#!/bin/bash
# round 6: config 5 on the KITTI blocks, the gradient tests under the two-run f64 envelope, the MFMA k_gd_proj;
# then the training step and the config-5 line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
export PCNERF_PARITY_REPORT=gpurun_out/r6b_report.jsonl
rm -f $PCNERF_PARITY_REPORT
timeout -k 10 700 python -u -m pytest tests/test_configs_gpu.py tests/test_backward_gpu.py tests/test_eval_driver.py -k "config5 or grads or view" -v --timeout 300 --timeout-method thread > gpurun_out/r6b_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6b_tests.log; echo "tests rc=$rc"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for v in 1 0 1 0; do   # layer 1's launch with dW_0's encoding columns fused (1, default) or k_wgrad_enc (0)
  PCNERF_REMAT_FUSE0=$v timeout -k 10 300 python3 bench.py --mode train_step --steps 10 --warmup 3 --no-extra --no-ceiling --no-cpu-baseline --no-fp32-line --detail gpurun_out/r6b_ts_f$v.detail.json > gpurun_out/r6b_ts_f$v.json 2> gpurun_out/r6b_ts_f$v.err
  rc=$?; echo "train_step fuse0=$v rc=$rc $(cut -c1-200 gpurun_out/r6b_ts_f$v.json)"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python3 bench.py --config 5 --steps 5 --warmup 2 --no-ceiling --detail gpurun_out/r6b_c5.detail.json > gpurun_out/r6b_c5.json 2> gpurun_out/r6b_c5.err
rc=$?; echo "config5 rc=$rc $(cut -c1-300 gpurun_out/r6b_c5.json)"
exit $rc
