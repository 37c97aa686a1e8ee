#!/bin/bash
# round 6: the config-5 test, a same-process A/B of the W waves' constants in registers (kreg1) or LDS (kreg0),
# then profiles of the eval / forward-only lines (TAG r06d)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
export PCNERF_PARITY_REPORT=gpurun_out/r6d_report.jsonl
rm -f $PCNERF_PARITY_REPORT
timeout -k 10 300 python -u -m pytest tests/test_configs_gpu.py -k "config5" -v --timeout 280 --timeout-method thread > gpurun_out/r6d_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6d_tests.log; echo "tests rc=$rc"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 400 python3 scripts/lib_ab.py kreg1 kreg0 --steps 5 --rounds 3 > gpurun_out/r6d_kreg_ab.txt 2>&1
rc=$?; cat gpurun_out/r6d_kreg_ab.txt; [ $rc -ne 0 ] && exit $rc
TAG=r06d LINES="val view config4 config5" bash scripts/gpu_profiles.sh
