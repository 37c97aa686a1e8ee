# PMC passes over a small training step (8,192 rays: 16 BatchNorm chunks) for the backward kernels; each pass its
# own rocprofv3 run (MI355X_MICROARCH slot limits), compacted per kernel.  usage: bash scripts/gpu_pmc_bwd.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-fb}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
ARGS="--mode train_step --rays 8192 --steps 1 --warmup 1 --no-extra --no-ceiling --no-fp32-line --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py $ARGS > $OUT/stats.json 2> $OUT/stats.err
rc=$?; echo "stats rc=$rc"; [ $rc -ne 0 ] && exit $rc
rm -f $OUT/stats/*kernel_trace.csv
for C in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_VMEM SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU" FETCH_SIZE WRITE_SIZE; do
  N=$(echo $C | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$N -o run -- python3 bench.py $ARGS > $OUT/pmc_$N.json 2> $OUT/pmc_$N.err
  rc=$?; echo "pmc $N rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 scripts/compact_pmc.py $OUT/pmc_$N
done
python3 - "$OUT" <<'PY'
import csv, glob, sys
out = sys.argv[1]
rows = {}
for f in glob.glob(out + "/pmc_*/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "bwd_fused" in r["Kernel_Name"] or "wgrad_b3" in r["Kernel_Name"] or "k_out_bwd" in r["Kernel_Name"]:
            rows.setdefault(r["Kernel_Name"][:60], {})[r["Counter_Name"]] = float(r["Counter_Value"])
for k, v in rows.items():
    print(k)
    for c, x in sorted(v.items()):
        print(f"   {c:28s} {x:.4g}")
    if "GRBM_GUI_ACTIVE" in v and "SQ_VALU_MFMA_BUSY_CYCLES" in v:
        print("   MfmaUtil %", 100 * v["SQ_VALU_MFMA_BUSY_CYCLES"] / (v["GRBM_GUI_ACTIVE"] * 256 * 4))
for f in glob.glob(out + "/stats/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "bwd_fused" in r["Name"] or "wgrad" in r["Name"] or "out_bwd" in r["Name"]:
            print(r["Name"][:50], r["Calls"], r["AverageNs"])
PY
