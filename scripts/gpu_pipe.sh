# split-mix micro check, fused-query A/B of the variant libraries, then the fused train-query parity tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/micro/split_mix > gpurun_out/split_mix.json 2>&1
rc=$?; cat gpurun_out/split_mix.json; echo "split_mix rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/fused_ab.py > gpurun_out/fused_ab.json 2> gpurun_out/fused_ab.err
rc=$?; cat gpurun_out/fused_ab.json; tail -3 gpurun_out/fused_ab.err; echo "ab rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_configs_gpu.py -m gpu -k "${TESTK:-fused}" -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_pipe.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_pipe.log; echo "tests rc=$rc"
exit $rc
