export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_eval_driver.py tests/test_eval_fold.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "eval or val or view or render_rays or config1 or config5" > gpurun_out/pytest_eval.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_eval.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --mode val --steps 5 --warmup 2 > gpurun_out/bench_valh.json 2> gpurun_out/bench_valh.err &&
timeout -k 10 300 python bench.py --mode view --steps 5 --warmup 2 > gpurun_out/bench_viewh.json 2> gpurun_out/bench_viewh.err &&
timeout -k 10 400 python bench.py --config 5 --steps 2 --warmup 1 > gpurun_out/bench_config5h.json 2> gpurun_out/bench_config5h.err
echo rc=$?
