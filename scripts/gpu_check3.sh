# full GPU suite + default bench (train_fwd) + rocprofv3 stats/PMC of train_step at this commit
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_tests.sh
rc=$?; echo "tests rc=$rc"
timeout -k 10 400 python bench.py > gpurun_out/bench_train_fwd.json 2> gpurun_out/bench_train_fwd.err
rc2=$?; echo "bench rc=$rc2"; [ $rc2 -ne 0 ] && exit $rc2
python3 -c "import json; d=json.load(open('gpurun_out/bench_train_fwd.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
bash scripts/profile.sh ${PROF_TAG:-r03e_train_step} --mode train_step --steps 3 --warmup 1
rc3=$?; echo "prof rc=$rc3"
exit $(( rc | rc3 ))
