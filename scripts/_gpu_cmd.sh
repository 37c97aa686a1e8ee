export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_last.json 2> gpurun_out/bench_last.err
echo rc=$?
