# All bench lines of the round (each step under its own time limit; stops at the first failure).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/bench
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/bench/$n.json 2> gpurun_out/bench/$n.err; rc=$?;
        echo "$n rc=$rc"; tail -c 400 gpurun_out/bench/$n.json; echo; return $rc; }
run train_fwd --steps 5 --warmup 2 &&
run val --mode val --steps 5 --warmup 2 &&
run view --mode view --steps 5 --warmup 2 &&
run train_step --mode train_step --steps 3 --warmup 1 &&
run train_step_refcfg --mode train_step --rays 256 --samples 768 --importance 1536 --steps 10 --warmup 2 --cpu-rays 32
