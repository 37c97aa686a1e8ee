# k_nof_eval_h2 A/B stamps of the variant libraries (eval and train instantiations)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/eh2c
for V in ${VARS:-stamp sl}; do for TRN in 0 1; do
  EH_TRAIN=$TRN timeout -k 10 120 python scripts/eh2_phases.py pc-nerf_amd/lib/variants/libpcnerf_$V.so > gpurun_out/eh2c/${V}_$TRN.json 2> gpurun_out/eh2c/${V}_$TRN.err
  rc=$?; echo "$V $TRN rc=$rc"; cut -c1-420 gpurun_out/eh2c/${V}_$TRN.json; [ $rc -ne 0 ] && exit $rc
done; done
exit 0
