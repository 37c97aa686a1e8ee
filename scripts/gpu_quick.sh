# quick GPU check: selected tests (TESTS env, pytest -k expression or node ids) + an optional bench line (BENCH env)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests -m gpu} -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_quick.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python bench.py $BENCH > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
  rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 -c "import json; d=json.load(open('gpurun_out/bench_quick.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
fi
exit 0
