# full GPU suite + default bench (train_fwd) + val bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_tests.sh -x
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_train_fwd.json 2> gpurun_out/bench_train_fwd.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 -c "import json; d=json.load(open('gpurun_out/bench_train_fwd.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['fp32_mfma']['value'], d['cpu_baseline']['value'])"
timeout -k 10 400 python bench.py --mode val > gpurun_out/bench_val.json 2> gpurun_out/bench_val.err
rc=$?; echo "val rc=$rc"; python3 -c "import json; d=json.load(open('gpurun_out/bench_val.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
exit $rc
