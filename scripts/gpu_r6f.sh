#!/bin/bash
# round 6: timing-only ablations of k_bwd_remat3<true> (abl1: W waves idle, abl2: D waves without MFMAs, abl3: D's
# B operands from registers), same-process step A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 scripts/lib_ab.py ${ABL_NAMES:-abl0 abl1 abl2 abl3} --steps 5 --rounds 2 > gpurun_out/r6f_abl.txt 2>&1
rc=$?; cat gpurun_out/r6f_abl.txt; exit $rc
