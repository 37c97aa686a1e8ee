set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ldspmc
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS --output-format csv -d gpurun_out/ldspmc -o run -- ./scripts/micro/lds_fb > gpurun_out/ldspmc/out.txt 2>&1
rc=$?
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/ldspmc/**/*counter_collection.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    by = {}
    for r in rows:
        by.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    for d in sorted(by):
        v = by[d]
        print(d, {k: round(x) for k, x in v.items()}, "conflict/instr %.2f" % (v["SQ_LDS_BANK_CONFLICT"] / max(v["SQ_INSTS_LDS"], 1)))
PY
exit $rc
