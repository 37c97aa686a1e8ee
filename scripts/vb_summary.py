"""Compact table of a variant_bench.py JSON output (per variant: median us of each kernel tag, diff vs base)."""
import json
import sys

txt = open(sys.argv[1]).read()
d = json.loads(txt[txt.index("{"):])
for name, v in d.items():
    row = " ".join(f"{k}={x['us']}" for k, x in v.items() if isinstance(x, dict) and "us" in x)
    if "clock_stamps" in v:
        row += " " + " ".join(f"{k}={x}" for k, x in v["clock_stamps"].items())
    print(f"{name:12s} {row} diff={v.get('max_rel_diff_vs_base', '-'):.3g}" if "max_rel_diff_vs_base" in v
          else f"{name:12s} {row}")
