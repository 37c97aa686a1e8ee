#!/bin/bash
# round 6: the encoding's sines / cosines by one float64 argument reduction per coordinate (enc_sincos.h) vs the
# library's sincosf per frequency: micro-benchmark, then same-process A/Bs of the headline forward and the step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/micro/enc_sincos_bench > gpurun_out/r6h_micro.txt 2>&1
rc=$?; cat gpurun_out/r6h_micro.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 scripts/lib_ab.py encnew enclib --fwd --steps 10 --rounds 3 > gpurun_out/r6h_fwd.txt 2>&1
rc=$?; cat gpurun_out/r6h_fwd.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 scripts/lib_ab.py encnew enclib --steps 5 --rounds 2 > gpurun_out/r6h_step.txt 2>&1
rc=$?; cat gpurun_out/r6h_step.txt; exit $rc
