#!/bin/bash
# round 6: the backward tests (k_bwd_remat3 and remat2), the new resample / eval-shell cases, then a train_step
# A/B of the two layer kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_backward_gpu.py tests/test_parity_gpu.py -k "grads or resample or eval_shell" -x -v --timeout 300 --timeout-method thread > gpurun_out/r6a_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r6a_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
for v in 3 2 3; do
  PCNERF_REMAT_VER=$v timeout -k 10 300 python3 bench.py --mode train_step --steps 10 --warmup 3 --no-extra --no-ceiling --no-cpu-baseline --no-fp32-line --detail gpurun_out/r6a_ts_v$v.detail.json > gpurun_out/r6a_ts_v$v.json 2> gpurun_out/r6a_ts_v$v.err
  rc=$?; echo "v$v rc=$rc $(cut -c1-300 gpurun_out/r6a_ts_v$v.json)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
