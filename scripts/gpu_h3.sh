# full GPU suite (parity report) + the default bench line + the val line + the training step, at this commit
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_tests.sh
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
mkdir -p gpurun_out/h3
for M in train_fwd val train_step; do
  timeout -k 10 400 python bench.py --mode $M > gpurun_out/h3/bench_$M.json 2> gpurun_out/h3/bench_$M.err
  rc=$?; echo "$M rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 -c "
import json
for n in ('train_fwd','val','train_step'):
    d=json.load(open('gpurun_out/h3/bench_'+n+'.json')); print(n, d['value'], d['ms_per_step'], d['kernels_step_ms'], round(sum(v['ms_per_step'] for v in d['kernels'].values()),3), d['roofline']['frac'])"
