# fused train query + per-element gradient parity: parity/config tests (fused math), backward tests, a bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
export PCNERF_PARITY_REPORT=gpurun_out/parity_report_fused.jsonl
rm -f $PCNERF_PARITY_REPORT
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_backward_gpu.py -m gpu -v --timeout 300 --timeout-method thread -k "fused or backward or grads" > gpurun_out/pytest_fused.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_fused.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
PCNERF_TRAIN_MATH=f16x2_3_fused timeout -k 10 400 python bench.py --no-fp32-line > gpurun_out/bench_fused.json 2> gpurun_out/bench_fused.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_fused.err; exit $rc
