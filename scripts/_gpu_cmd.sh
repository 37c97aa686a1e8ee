export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "eval or val or view or render_rays" > gpurun_out/pytest_eval.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_eval.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --mode val --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_valh.json 2> gpurun_out/bench_valh.err &&
timeout -k 10 300 python bench.py --mode view --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_viewh.json 2> gpurun_out/bench_viewh.err
echo rc=$?
