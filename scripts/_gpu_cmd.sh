export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_tests.sh && LINES="val view view_frame config5" bash scripts/gpu_bench_all.sh r02i
echo rc=$?
