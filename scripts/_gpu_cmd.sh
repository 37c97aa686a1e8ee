export TMPDIR=/tmp
mkdir -p gpurun_out
VB_BWD=0 timeout -k 10 300 python scripts/variant_bench.py > gpurun_out/vb_eh2.json 2> gpurun_out/vb_eh2.err
echo vb rc=$?
rm -rf pc-nerf_amd/lib/variants
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "eval or val or view or render_rays" > gpurun_out/pytest_eval.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_eval.log; exit $rc
