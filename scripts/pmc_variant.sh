# One PMC pass over scripts/variant_bench.py for the given variants; summary via scripts/pmc_kernels.py
# usage: bash scripts/pmc_variant.sh <tag> <variant,variant> ["COUNTERS"]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; V=$2
C=${3:-"SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY"}
OUT=gpurun_out/pmcv/$TAG
mkdir -p $OUT
VB_BWD=${VB_BWD:-0} VB_ONLY=$V timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT -o run -- \
  python3 scripts/variant_bench.py > $OUT/vb.json 2> $OUT/vb.err
rc=$?; echo "pmc $TAG rc=$rc"; exit $rc
