# k_nof_eval_h2 rework: parity (eval + fused train) and phase stamps of both instantiations
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/eh2b
export PCNERF_PARITY_REPORT=gpurun_out/eh2b/parity.jsonl
rm -f $PCNERF_PARITY_REPORT
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_eval_driver.py -m gpu -v --timeout 300 --timeout-method thread -k "not fp32 and not f16x2_3-" > gpurun_out/eh2b/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/eh2b/pytest.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for TRN in 0 1; do
  EH_TRAIN=$TRN timeout -k 10 120 python scripts/eh2_phases.py pc-nerf_amd/lib/variants/libpcnerf_stamp.so > gpurun_out/eh2b/stamp_$TRN.json 2> gpurun_out/eh2b/stamp_$TRN.err
  rc=$?; echo "stamp $TRN rc=$rc"; cat gpurun_out/eh2b/stamp_$TRN.json; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python bench.py --no-fp32-line > gpurun_out/eh2b/bench.json 2> gpurun_out/eh2b/bench.err
rc=$?; echo "bench rc=$rc"; python3 -c "import json; d=json.load(open('gpurun_out/eh2b/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cd_vs_ref'])"
exit $rc
