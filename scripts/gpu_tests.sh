#!/bin/bash
# GPU test suite with the parity report (tests/test_configs_gpu.py writes one JSON line per config).
set -o pipefail
mkdir -p gpurun_out
export PCNERF_PARITY_REPORT=gpurun_out/parity_report.jsonl
export PCNERF_PARITY_DUMP=gpurun_out/config2_full_hip.npz
rm -f "$PCNERF_PARITY_REPORT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
exit $rc
