# fused-query A/B of the variant libraries (VB_ONLY) + phase stamps of the stamp variants (STAMPS)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
if [ "$VB_ONLY" != "none" ]; then
  timeout -k 10 300 python -u scripts/fused_ab.py > gpurun_out/ab/fused_ab.json 2> gpurun_out/ab/fused_ab.err
  rc=$?; cat gpurun_out/ab/fused_ab.json; echo "ab rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
for V in $STAMPS; do for TRN in ${STRAIN:-1}; do
  EH_TRAIN=$TRN timeout -k 10 120 python scripts/eh2_phases.py pc-nerf_amd/lib/variants/libpcnerf_$V.so > gpurun_out/ab/${V}_$TRN.json 2> gpurun_out/ab/${V}_$TRN.err
  rc=$?; echo "$V $TRN rc=$rc"; cat gpurun_out/ab/${V}_$TRN.json; [ $rc -ne 0 ] && exit $rc
done; done
exit 0
