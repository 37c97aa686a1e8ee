set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash scripts/gpu_tests.sh -k "depth2 or render_rays or test_abi" && \
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?
tail -c 3000 gpurun_out/bench_default.json
exit $rc
