# fused-query A/B of the variant libraries, then selected GPU tests (TESTK pytest -k expression) on the main library
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u scripts/fused_ab.py > gpurun_out/ab/fused_ab.json 2> gpurun_out/ab/fused_ab.err
rc=$?; cat gpurun_out/ab/fused_ab.json; tail -3 gpurun_out/ab/fused_ab.err; echo "ab rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u -m pytest ${TESTF:-tests/test_parity_gpu.py tests/test_configs_gpu.py} -m gpu -k "${TESTK:-fused}" -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_abt.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_abt.log | tail -30; tail -3 gpurun_out/pytest_abt.log; echo "tests rc=$rc"
exit $rc
