set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcv
rocprofv3 -L > gpurun_out/pmcv/counters.txt 2>&1 || true
bash scripts/pmc_variant.sh h1 base "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" &&
bash scripts/pmc_variant.sh h2 base "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE" &&
bash scripts/pmc_variant.sh h3 base "FETCH_SIZE" && bash scripts/pmc_variant.sh h4 base "WRITE_SIZE"
