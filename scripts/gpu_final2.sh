# full GPU suite (parity report) + rocprofv3 stats / PMC passes of the train_step line at this commit
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r03k}
bash scripts/gpu_tests.sh
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash scripts/profile.sh ${TAG}_train_step --mode train_step --steps 2 --warmup 1
rc2=$?; echo "prof rc=$rc2"
exit $(( rc | rc2 ))
