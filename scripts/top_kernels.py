"""Per-step kernel table of a profile.sh stats pass: python scripts/top_kernels.py <tag> [steps] [n]"""
import csv
import re
import sys


def short(name):
    m = re.match(r"_ZN3pcn(\d+)", name)
    if not m:
        return name.split("(")[0].replace("void ", "").replace("pcn::", "")
    i, n = m.end(), int(m.group(1))
    ident, i = name[i:i + n], i + n
    if i < len(name) and name[i] == "I":
        args = re.findall(r"L([ib])(\d+)E", name[i + 1:name.find("EE", i) + 1])
        ident += "<" + ",".join(("true" if v == "1" else "false") if t == "b" else v for t, v in args) + ">"
    return ident


tag = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 7.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows = list(csv.DictReader(open(f"gpurun_out/prof/{tag}/stats/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"all kernels: {tot / 1e6 / steps:.3f} ms per step ({steps:g} steps)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print(f"{short(r['Name'])[:56]:56s} {int(r['Calls']) / steps:6.1f}/step {float(r['AverageNs']) / 1e3:9.2f} us "
          f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms/step")
