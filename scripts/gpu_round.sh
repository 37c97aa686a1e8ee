# One GPU call: bench lines for every mode/config, then rocprofv3 stats + PMC passes for the headline (train_fwd)
# and the training step.   usage: bash scripts/gpu_round.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r02}
bash scripts/gpu_bench_all.sh $TAG &&
bash scripts/profile.sh ${TAG}_train_fwd --steps 5 --warmup 2 &&
bash scripts/profile.sh ${TAG}_train_step --mode train_step --steps 2 --warmup 1
