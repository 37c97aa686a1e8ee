export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_tests.sh &&
timeout -k 10 300 python bench.py > gpurun_out/bench_gram5.json 2> gpurun_out/bench_gram5.err &&
bash scripts/profile.sh r02g_train_fwd --steps 5 --warmup 2
echo rc=$?
