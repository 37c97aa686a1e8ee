# Forward occupancy experiment: the store-writing train query and the eval query of variant
# libraries built with EH3_SB / EH3_WG_PER_CU of csrc/nof_eval.hip set per variant (base: 6 sample blocks, one block
# per CU; sb3x2: 3 sample blocks, two blocks per CU -- adopted; sb3x1: 3 sample blocks, one block per CU; the run in
# profiles/r04_occupancy_* used -D macros for the two constants) -- same-process A/B, then one PMC pass per variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/occ
FA_STORE=1 FA_RAYS=65536 FA_S=384 timeout -k 10 400 python3 -u scripts/fused_ab.py > gpurun_out/occ/ab.json \
  2> gpurun_out/occ/ab.err
rc=$?; cat gpurun_out/occ/ab.json; [ $rc -ne 0 ] && exit $rc
for v in base sb3x2; do
  VB_ONLY=$v FA_ROUNDS=2 FA_STORE=1 FA_RAYS=65536 FA_S=384 timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES \
    GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_ANY SQ_INSTS_LDS \
    --output-format csv -d gpurun_out/occ/pmc_$v -o run -- python3 scripts/fused_ab.py > gpurun_out/occ/pmc_$v.out \
    2> gpurun_out/occ/pmc_$v.err
  rc=$?; echo "pmc $v rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 scripts/compact_pmc.py gpurun_out/occ/pmc_$v
done
exit 0
