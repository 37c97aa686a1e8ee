#!/bin/bash
# round 6: new tests (composite workgroup per ray, torch ops, eval-shell resample, small-chunk gradients with a
# report), then a train_step A/B of k_bwd_remat3 / remat2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
export PCNERF_PARITY_REPORT=gpurun_out/r6a_small_report.jsonl
rm -f $PCNERF_PARITY_REPORT
timeout -k 10 600 python -u -m pytest tests/test_torch_ops.py tests/test_backward_gpu.py tests/test_parity_gpu.py -k "torch or grads or resample or eval_shell or workgroup" -v --timeout 300 --timeout-method thread > gpurun_out/r6a_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6a_tests.log; echo "tests rc=$rc"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for v in 3 4 2 3 4; do
  PCNERF_REMAT_VER=$v timeout -k 10 300 python3 bench.py --mode train_step --steps 10 --warmup 3 --no-extra --no-ceiling --no-cpu-baseline --no-fp32-line --detail gpurun_out/r6a_ts_v$v.detail.json > gpurun_out/r6a_ts_v$v.json 2> gpurun_out/r6a_ts_v$v.err
  rc=$?; echo "v$v rc=$rc $(cut -c1-200 gpurun_out/r6a_ts_v$v.json)"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python3 bench.py --mode train_step --rays 256 --samples 768 --importance 1536 --steps 10 --warmup 3 --no-extra --no-ceiling --no-cpu-baseline --no-fp32-line --detail gpurun_out/r6a_ref.detail.json > gpurun_out/r6a_ref.json 2> gpurun_out/r6a_ref.err
rc=$?; echo "refcfg rc=$rc $(cut -c1-200 gpurun_out/r6a_ref.json)"
exit $rc
