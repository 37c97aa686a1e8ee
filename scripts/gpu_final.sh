# Round-end check at HEAD: the full GPU suite + smoke() + the default bench (scripts/gpu_default.sh), then the
# train_step rocprofv3 stats + PMC passes (TAG, default r04g)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_default.sh || exit $?
bash scripts/profile.sh ${TAG:-r04g}_train_step --mode train_step --steps 2 --warmup 1 --no-ceiling
rc=$?; echo "prof rc=$rc"; exit $rc
