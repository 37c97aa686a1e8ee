# rocprofv3 stats + PMC passes of the headline (train_fwd) and val at this commit
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/profile.sh r03d_train_fwd --steps 5 --warmup 2 && bash scripts/profile.sh r03d_val --mode val --steps 3 --warmup 1
