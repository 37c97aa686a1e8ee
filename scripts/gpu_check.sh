set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-rays 256 --mode ${BENCH_MODE:-train_fwd} > gpurun_out/bench1.json 2> gpurun_out/bench1.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench1.json; tail -5 gpurun_out/bench1.err
exit $rc
