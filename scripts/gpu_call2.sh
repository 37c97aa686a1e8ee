# One GPU call: the backward tests (pytest -k $K), then a short train_step bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PCNERF_PARITY_REPORT=gpurun_out/parity_report.jsonl
rm -f "$PCNERF_PARITY_REPORT"
timeout -k 10 600 python -u -m pytest tests/test_backward_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "${K:-fused}" > gpurun_out/pytest_bwd.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_bwd.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --mode train_step --steps 5 --warmup 2 --no-extra --no-ceiling --no-fp32-line --no-cpu-baseline > gpurun_out/bench_ts.json 2> gpurun_out/bench_ts.err
rc2=$?
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench_ts.json"))
print("train_step", d["value"], d["ms_per_step"])
for k, v in d["kernels"].items(): print(k, v["kernel"], v["ms_per_step"], v["launches_per_step"], v["avg_us"], v["GB/s"])
PY
exit $(( rc > rc2 ? rc : rc2 ))
