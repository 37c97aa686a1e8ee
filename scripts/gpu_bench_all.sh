# All bench lines of the round (each step under its own time limit; stops at the first failure).
# usage: bash scripts/gpu_bench_all.sh <tag>   -> gpurun_out/bench/<tag>_<line>.json
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r02}
mkdir -p gpurun_out/bench
if [ -n "$LINES" ]; then   # a subset: LINES="train_fwd val ..."
  for l in $LINES; do grep -q "^run $l " $0 || { echo "unknown line $l"; exit 2; }; done
fi
want() { [ -z "$LINES" ] || [[ " $LINES " == *" $1 "* ]]; }
run() { n=$1; want $n || return 0; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/bench/${TAG}_$n.json 2> gpurun_out/bench/${TAG}_$n.err; rc=$?;
        echo "$n rc=$rc"; tail -c 300 gpurun_out/bench/${TAG}_$n.json; echo; return $rc; }
run train_fwd --steps 20 --warmup 5 &&
run val --mode val --steps 5 --warmup 2 &&
run view --mode view --steps 5 --warmup 2 &&
run view_frame --mode view --rays 101000 --steps 3 --warmup 1 --cpu-rays 256 &&
run train_step --mode train_step --steps 3 --warmup 1 &&
run config3 --config 3 --steps 3 --warmup 1 &&
run config4 --config 4 --steps 2 --warmup 1 &&
run config5 --config 5 --steps 2 --warmup 1 &&
run val_fold --mode val --fold --steps 5 --warmup 2 &&
run view_fold --mode view --fold --steps 5 --warmup 2 &&
run train_step_refcfg --mode train_step --rays 256 --samples 768 --importance 1536 --steps 10 --warmup 2 --cpu-rays 32 &&
run train_fwd_fold --fold --steps 10 --warmup 2 &&
run train_step_fold --mode train_step --fold --steps 5 --warmup 1
