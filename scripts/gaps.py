"""Idle time between consecutive kernels of a rocprofv3 kernel trace (scripts/gap_trace.sh): python scripts/gaps.py
<tag> [last_ms]  -- over the trace's last ``last_ms`` ms (the timed steps), the total busy / idle time and the
kernels that follow the largest idle gaps."""
import collections
import csv
import glob
import sys

tag = sys.argv[1]
last_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 1e9
f = glob.glob(f"gpurun_out/trace/{tag}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f))))
t_end = rows[-1][1]
rows = [r for r in rows if r[0] >= t_end - last_ms * 1e6]
busy = idle = 0
by_next = collections.Counter()
cnt = collections.Counter()
prev_end = rows[0][0]
for s, e, n in rows:
    gap = max(0, s - prev_end)
    idle += gap
    short = n.split("(")[0].replace("void ", "")[:60]
    by_next[short] += gap
    cnt[short] += 1
    busy += e - max(s, prev_end) if e > prev_end else 0
    prev_end = max(prev_end, e)
span = rows[-1][1] - rows[0][0]
print(f"window {span / 1e6:.2f} ms: busy {busy / 1e6:.2f} ms, idle {idle / 1e6:.2f} ms, {len(rows)} kernels")
for k, v in by_next.most_common(15):
    print(f"  {v / 1e6:8.3f} ms idle before {cnt[k]:5d} x {k}")
