# usage: bash scripts/gpu_bench.sh [bench.py args...]   (runs the parity tests first; stops on a crash)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 400 python bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
exit $rc
