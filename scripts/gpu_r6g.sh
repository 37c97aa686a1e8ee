#!/bin/bash
# round 6: k_bwd_remat3 with eight W waves (PCNERF_REMAT_W8=1): the default-math gradient tests, then a same-process
# A/B against four W waves, each with / without the W waves' early transposed reads (WORDER 2)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
export PCNERF_PARITY_REPORT=gpurun_out/r6g_report.jsonl
rm -f $PCNERF_PARITY_REPORT
PCNERF_REMAT_W8=1 timeout -k 10 400 python -u -m pytest tests/test_backward_gpu.py -k "(f16x2_3_fused and not remat and not store) or large_chunks" -v --timeout 300 --timeout-method thread > gpurun_out/r6g_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6g_tests.log; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 scripts/lib_ab.py v0 wo2 w8 w8wo2 --steps 5 --rounds 3 > gpurun_out/r6g_ab.txt 2>&1
rc=$?; cat gpurun_out/r6g_ab.txt; exit $rc
