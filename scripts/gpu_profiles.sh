# rocprofv3 stats + PMC passes of every default bench line at this commit (TAG prefix; profiles/<TAG>_<line>_*)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r05h}
bash scripts/profile.sh ${TAG}_train_fwd --steps 3 --warmup 1 --no-extra --no-ceiling && \
bash scripts/profile.sh ${TAG}_val --mode val --steps 3 --warmup 1 --no-ceiling && \
bash scripts/profile.sh ${TAG}_view --mode view --steps 3 --warmup 1 --no-ceiling && \
bash scripts/profile.sh ${TAG}_train_step --mode train_step --steps 2 --warmup 1 --no-ceiling && \
bash scripts/profile.sh ${TAG}_train_step_refcfg --mode train_step --rays 256 --samples 768 --importance 1536 \
  --steps 5 --warmup 2 --no-ceiling && \
bash scripts/profile.sh ${TAG}_config3 --config 3 --mode train_step --rays 262144 --samples 64 --importance 128 \
  --steps 2 --warmup 1 --no-ceiling && \
bash scripts/profile.sh ${TAG}_config4 --config 4 --rays 262144 --samples 128 --importance 256 --steps 2 --warmup 1 \
  --no-ceiling
rc=$?; echo "prof rc=$rc"
exit $rc
