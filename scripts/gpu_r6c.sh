#!/bin/bash
# round 6: the config-5 test, the default bench run, then profiles of the training lines (TAG r06c)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
export PCNERF_PARITY_REPORT=gpurun_out/r6c_report.jsonl
rm -f $PCNERF_PARITY_REPORT
timeout -k 10 300 python -u -m pytest tests/test_configs_gpu.py -k "config5" -v --timeout 280 --timeout-method thread > gpurun_out/r6c_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6c_tests.log; echo "tests rc=$rc"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
TESTS=0 bash scripts/gpu_default.sh || exit $?
TAG=r06c LINES="train_fwd train_step train_step_refcfg config3" bash scripts/gpu_profiles.sh
