export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_tests.sh && timeout -k 10 300 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo rc=$?
