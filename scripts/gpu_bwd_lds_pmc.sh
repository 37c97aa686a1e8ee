# One PMC pass over a short training step for the fused backward's LDS use: LDS-array busy cycles, bank-conflict
# cycles, LDS instructions, against GPU-busy cycles (gpurun_out/bwdlds/)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/bwdlds
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAVES \
  SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/bwdlds/pmc -o run -- python3 bench.py \
  --mode train_step --rays 16384 --steps 1 --warmup 0 --no-extra --no-ceiling --no-fp32-line --no-cpu-baseline \
  > gpurun_out/bwdlds/out.json 2> gpurun_out/bwdlds/err.txt
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 scripts/compact_pmc.py gpurun_out/bwdlds/pmc
