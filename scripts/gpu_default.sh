# full GPU suite (parity report) + smoke() + the default bench run exactly as the driver runs it
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
if [ "$TESTS" != "0" ]; then
  bash scripts/gpu_tests.sh
  rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; tail -2 gpurun_out/smoke.log; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
s=$(date +%s)
timeout -k 10 600 python3 bench.py ${BENCH_ARGS} --detail gpurun_out/bench_default_detail.json > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; echo "bench rc=$rc wall=$(( $(date +%s) - s ))s"; exit $rc
