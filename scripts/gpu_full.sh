# full GPU suite (with the parity report) + the default bench line + the val line, at this commit
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_tests.sh
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_train_fwd.json 2> gpurun_out/bench_train_fwd.err
rc2=$?; echo "bench rc=$rc2"; [ $rc2 -ne 0 ] && exit $rc2
python3 -c "import json; d=json.load(open('gpurun_out/bench_train_fwd.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 400 python bench.py --mode val > gpurun_out/bench_val.json 2> gpurun_out/bench_val.err
rc3=$?; echo "val rc=$rc3"
python3 -c "import json; d=json.load(open('gpurun_out/bench_val.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
exit $(( rc | rc3 ))
