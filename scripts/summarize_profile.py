"""Summarise a scripts/profile.sh run (gpurun_out/prof/<tag>) into profiles/<tag>_*.

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section): FETCH_SIZE and WRITE_SIZE come
from separate PMC passes (KiB per dispatch); on gfx950 FETCH_SIZE reports exactly half the bytes of a wide
(16 B/lane) coalesced streaming read, so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for 16 B/lane
stores.  MfmaUtil = SQ_VALU_MFMA_BUSY_CYCLES / (per-XCD GRBM_GUI_ACTIVE x 1024 SIMDs)."""
import collections
import csv
import json
import os
import re
import shutil
import subprocess
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = os.path.join("gpurun_out", "prof", tag)
dst = "profiles"
os.makedirs(dst, exist_ok=True)


def demangle(name):
    """rocprofv3 leaves names with fp16/bf16 vector parameters mangled (and c++filt here cannot read them): the
    pcn:: kernel name and its integer / bool template arguments are all this needs."""
    m = re.match(r"_ZN3pcn(\d+)", name)
    if not m:
        return name
    i = m.end()
    n = int(m.group(1))
    ident, i = name[i:i + n], i + n
    if i < len(name) and name[i] == "I":
        args = re.findall(r"L([ib])(\d+)E", name[i + 1:name.find("EE", i) + 1])
        ident += "<" + ",".join(("true" if v == "1" else "false") if t == "b" else v for t, v in args) + ">"
    return "pcn::" + ident + "()"


def short(name):
    n = demangle(name).split("(")[0].replace("void ", "").replace("pcn::", "")
    return n.replace(" ", "")


stats = list(csv.DictReader(open(os.path.join(src, "stats", "run_kernel_stats.csv"))))
shutil.copy(os.path.join(src, "stats", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
pmc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sorted(os.listdir(src)):
    f = os.path.join(src, d, "run_counter_collection.csv")
    if d.startswith("pmc_") and os.path.exists(f):
        for r in csv.DictReader(open(f)):
            pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
summary = {}
for r in stats:
    k = short(r["Name"])
    e = {"calls": int(r["Calls"]), "avg_us": round(float(r["AverageNs"]) / 1e3, 2),
         "pct_time": round(float(r["Percentage"]), 2)}
    c = {n: sum(v) / len(v) for n, v in pmc.get(k, {}).items()}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        e["FETCH_SIZE_KiB"] = round(c["FETCH_SIZE"], 1)
        e["WRITE_SIZE_KiB"] = round(c["WRITE_SIZE"], 1)
        e["hbm_bytes_per_launch"] = int(2 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c and c["GRBM_GUI_ACTIVE"] > 0:
        e["MfmaUtil_pct"] = round(100 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024), 1)
        e["clock_GHz"] = round(c["GRBM_GUI_ACTIVE"] / 8 / (float(r["AverageNs"]) * 1e-9) / 1e9, 2)
    if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"] > 0:
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if n in c:
                e[n + "_pct"] = round(100 * c[n] / c["SQ_WAVE_CYCLES"], 1)
    summary[k] = e
with open(os.path.join(dst, f"{tag}_pmc_summary.json"), "w") as fh:
    json.dump(summary, fh, indent=1)
# profiles/pmc_traffic.json: HBM bytes per launch of the CURRENT kernels.  Each entry records the commit it was
# summarised at; entries of earlier commits are kept only while pc-nerf_amd/csrc is unchanged since then (so a
# kernel's bytes always describe the code at HEAD).  bench.py quotes the entry and its commit.
traffic_path = os.path.join(dst, "pmc_traffic.json")
traffic = json.load(open(traffic_path)) if os.path.exists(traffic_path) else {}
head = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True, text=True).stdout.strip()
meta = traffic.get("_meta", {})


def code_unchanged(since):
    return bool(since) and subprocess.run(["git", "diff", "--quiet", since, "HEAD", "--", "pc-nerf_amd/csrc"],
                                          capture_output=True).returncode == 0


kernels = {k: e for k, e in traffic.get("kernels", {}).items() if code_unchanged(e.get("head", meta.get("head")))}
for k, e in kernels.items():
    e.setdefault("head", meta.get("head"))
line = tag.split("_", 1)[1] if "_" in tag else None   # <prefix>_<bench line>, e.g. r04b_train_step
for k, e in summary.items():
    if "hbm_bytes_per_launch" in e:
        ent = {"hbm_bytes_per_launch": e["hbm_bytes_per_launch"], "avg_us": e["avg_us"], "profile": tag, "head": head}
        kernels[k] = ent
        if line:   # the same kernel can move different bytes in different lines (bench.py prefers this entry)
            kernels[f"{k}@{line}"] = dict(ent)
profs = sorted({e["profile"] for e in kernels.values()})
cmd = open(os.path.join(src, "command.txt")).read().strip() if os.path.exists(os.path.join(src, "command.txt")) else ""
cmds = {t: c for t, c in meta.get("commands", {}).items() if t in profs}
cmds[tag] = cmd
out = {"_meta": {"head": head, "profile": ",".join(profs), "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes "
                 "(scripts/profile.sh), bytes = 2 x FETCH_SIZE + WRITE_SIZE (gfx950 correction); each kernel "
                 "entry names the commit its profile was summarised at (pc-nerf_amd/csrc unchanged since)",
                 "commands": cmds},
       "kernels": kernels}
with open(traffic_path, "w") as fh:
    json.dump(out, fh, indent=1)
for k, e in list(summary.items())[:8]:
    print(k, e)
