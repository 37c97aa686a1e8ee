export TMPDIR=/tmp
mkdir -p gpurun_out
VB_BWD=0 timeout -k 10 300 python scripts/variant_bench.py > gpurun_out/vb_eh4.json 2> gpurun_out/vb_eh4.err
echo vb rc=$?
rm -rf pc-nerf_amd/lib/variants
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_eval_driver.py tests/test_eval_fold.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "eval or val or view or render_rays or config1 or config5" > gpurun_out/pytest_eval.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_eval.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --mode val --steps 5 --warmup 2 > gpurun_out/bench_valh2.json 2> gpurun_out/bench_valh2.err &&
timeout -k 10 300 python bench.py --mode view --steps 5 --warmup 2 > gpurun_out/bench_viewh2.json 2> gpurun_out/bench_viewh2.err
echo rc=$?
