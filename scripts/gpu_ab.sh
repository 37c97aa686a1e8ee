# fused-query A/B of the variant libraries (VB_ONLY)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
if [ "$VB_ONLY" != "none" ]; then
  timeout -k 10 300 python -u scripts/fused_ab.py > gpurun_out/ab/fused_ab.json 2> gpurun_out/ab/fused_ab.err
  rc=$?; cat gpurun_out/ab/fused_ab.json; echo "ab rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
exit 0
