"""Per-kernel averages of a rocprofv3 PMC csv (gpurun_out/pmcv/<tag>): MFMA busy %, clock, wait fractions."""
import collections
import csv
import glob
import sys

rows = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"gpurun_out/pmcv/{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pcn::", "")
        rows[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in rows.items():
    a = {n: sum(v) / len(v) for n, v in c.items()}
    out = [f"{k[:40]:40s} n={len(next(iter(c.values())))}"]
    if "SQ_VALU_MFMA_BUSY_CYCLES" in a and a.get("GRBM_GUI_ACTIVE"):
        out.append(f"mfma={100 * a['SQ_VALU_MFMA_BUSY_CYCLES'] / (a['GRBM_GUI_ACTIVE'] / 8 * 1024):.1f}%")
        out.append(f"gui_cyc={a['GRBM_GUI_ACTIVE'] / 8:.0f}")
    if a.get("SQ_WAVE_CYCLES"):
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if n in a:
                out.append(f"{n[3:]}={100 * a[n] / a['SQ_WAVE_CYCLES']:.1f}%")
    print(" ".join(out))
if len(sys.argv) > 2:   # raw per-launch averages of every counter for kernels whose name contains argv[2]
    for k, c in rows.items():
        if sys.argv[2] in k:
            print(k[:60], {n: round(sum(v) / len(v)) for n, v in sorted(c.items())})
