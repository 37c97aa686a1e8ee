# fused query + activation store: backward / config tests, then train_step under the layered and the fused forward
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/fs
timeout -k 10 900 python -u -m pytest tests/test_backward_gpu.py tests/test_configs_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/fs/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR" gpurun_out/fs/pytest.log | tail -45; tail -3 gpurun_out/fs/pytest.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
for M in f16x2_3 f16x2_3_fused; do
  PCNERF_TRAIN_MATH=$M timeout -k 10 400 python bench.py --mode train_step --steps 3 --warmup 1 --no-cpu-baseline --no-fp32-line > gpurun_out/fs/ts_$M.json 2> gpurun_out/fs/ts_$M.err
  rc=$?; echo "$M rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 -c "import json; d=json.load(open('gpurun_out/fs/ts_$M.json')); print('$M', d['value'], d['ms_per_step'], d['train_math'], {k: v['ms_per_step'] for k, v in d['kernels'].items()})"
done
exit 0
