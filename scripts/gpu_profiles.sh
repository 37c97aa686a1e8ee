# rocprofv3 stats + PMC passes of the train_fwd, val and train_step lines at this commit (TAG prefix)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r03m}
bash scripts/profile.sh ${TAG}_train_fwd --steps 3 --warmup 1 --no-extra --no-ceiling && \
bash scripts/profile.sh ${TAG}_val --mode val --steps 3 --warmup 1 --no-ceiling && \
bash scripts/profile.sh ${TAG}_train_step --mode train_step --steps 2 --warmup 1 --no-ceiling
rc=$?; echo "prof rc=$rc"
exit $rc
