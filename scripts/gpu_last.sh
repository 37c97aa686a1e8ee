# smoke() + the default bench line + the val line at this commit
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/last
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/last/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/last/smoke.log; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/last/bench_train_fwd.json 2> gpurun_out/last/bench_train_fwd.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --mode val > gpurun_out/last/bench_val.json 2> gpurun_out/last/bench_val.err
rc=$?; echo "val rc=$rc"
python3 -c "
import json
for n in ('train_fwd','val'):
    d=json.load(open('gpurun_out/last/bench_'+n+'.json')); print(n, d['value'], d['ms_per_step'], d['kernels_step_ms'], round(sum(v['ms_per_step'] for v in d['kernels'].values()),3), d['roofline']['frac'])"
exit $rc
