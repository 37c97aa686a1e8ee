# One GPU call: selected GPU tests (args to pytest -k), then the default bench line (all extra lines).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash scripts/gpu_tests.sh -k "${K:-depth2 or render_rays or test_abi}"
rc=$?
# pytest's exit codes 0 (passed) and 1 (tests failed) leave the GPU usable; anything else ends the call here
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc2=$?
tail -c 1500 gpurun_out/bench_default.json
tail -5 gpurun_out/bench_default.err
exit $(( rc > rc2 ? rc : rc2 ))
