# rocprofv3 stats + PMC passes of the default bench lines at this commit (TAG prefix; profiles/<TAG>_<line>_*)
# LINES: a subset, e.g. LINES="train_fwd train_step" (default: all eight)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r05h}
LINES=${LINES:-"train_fwd val view train_step train_step_refcfg config3 config4 config5"}
for ln in $LINES; do
  case $ln in
    train_fwd) args="--steps 3 --warmup 1 --no-extra --no-ceiling" ;;
    val) args="--mode val --steps 3 --warmup 1 --no-ceiling" ;;
    view) args="--mode view --steps 3 --warmup 1 --no-ceiling" ;;
    train_step) args="--mode train_step --steps 2 --warmup 1 --no-ceiling" ;;
    train_step_refcfg) args="--mode train_step --rays 256 --samples 768 --importance 1536 --steps 5 --warmup 2 --no-ceiling" ;;
    config3) args="--config 3 --mode train_step --rays 262144 --samples 64 --importance 128 --steps 2 --warmup 1 --no-ceiling" ;;
    config4) args="--config 4 --rays 262144 --samples 128 --importance 256 --steps 2 --warmup 1 --no-ceiling" ;;
    config5) args="--config 5 --steps 3 --warmup 1 --no-ceiling" ;;
    *) echo "unknown line $ln"; exit 2 ;;
  esac
  bash scripts/profile.sh ${TAG}_$ln $args
  rc=$?; echo "prof $ln rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
