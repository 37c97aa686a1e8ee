# full GPU suite (parity report) + smoke() + the bench lines named in LINES (scripts/gpu_bench_all.sh; TESTS=0 skips the first two)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r03n}
if [ "$TESTS" != "0" ]; then
  bash scripts/gpu_tests.sh
  rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; tail -2 gpurun_out/smoke.log; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
bash scripts/gpu_bench_all.sh $TAG
