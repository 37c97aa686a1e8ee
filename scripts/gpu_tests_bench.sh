#!/bin/bash
# GPU test suite (scripts/gpu_tests.sh), then one training-step bench line (gpurun_out/bench_ts.json)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_tests.sh "$@" || exit $?
timeout -k 10 300 python3 bench.py --mode train_step --steps 5 --warmup 2 --no-extra --no-ceiling --no-cpu-baseline \
  --no-fp32-line > gpurun_out/bench_ts.json 2> gpurun_out/bench_ts.err
rc=$?; tail -c 600 gpurun_out/bench_ts.json; exit $rc
