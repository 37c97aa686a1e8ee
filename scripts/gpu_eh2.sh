# k_nof_eval_h2 diagnostics: phase stamps (variant build) + PMC passes of the plain library on the same workload
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/eh2
timeout -k 10 120 python scripts/eh2_phases.py pc-nerf_amd/lib/variants/libpcnerf_stamp.so > gpurun_out/eh2/stamp.json 2> gpurun_out/eh2/stamp.err
rc=$?; echo "stamp rc=$rc"; cat gpurun_out/eh2/stamp.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/eh2_phases.py > gpurun_out/eh2/plain.json 2> gpurun_out/eh2/plain.err
rc=$?; echo "plain rc=$rc"; cat gpurun_out/eh2/plain.json; [ $rc -ne 0 ] && exit $rc
export EH_RAYS=4096 EH_WARM=0.1 EH_REPS=2
for C in "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_REQ_sum" \
         "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_VMEM SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"; do
  N=$(echo $C | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/eh2/pmc_$N -o run -- python3 scripts/eh2_phases.py > gpurun_out/eh2/pmc_$N.json 2> gpurun_out/eh2/pmc_$N.err
  rc=$?; echo "pmc $N rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 scripts/compact_pmc.py gpurun_out/eh2/pmc_$N
done
exit 0
