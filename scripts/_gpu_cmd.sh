export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_tests.sh
echo rc=$?
