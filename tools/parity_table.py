"""Reduce a GS_PARITY_REPORT file (tests/parity_report.py) to the DESIGN.md parity table: per test
(parametrisations folded) and tensor group, the bound asserted and the measured maxima.
usage: python tools/parity_table.py gpurun_out/parity.jsonl > profiles/rNN_parity_table.md"""
import collections
import json
import re
import sys

CHAIN = {"dmeans3D", "dscales", "drotations", "dcov3D", "dmeans2D"}
rows = collections.OrderedDict()
for line in open(sys.argv[1]):
    r = json.loads(line)
    test = re.sub(r"\[.*\]$", "", r["test"])  # fold the parametrisations
    tensor = r["tensor"].split(" (")[0]
    group = "image" if tensor in ("image", "color") else ("chain" if tensor in CHAIN else "other")
    key = (test, tensor, r["rtol"], r["frac"])
    a = rows.setdefault(key, dict(n=0, frac=0.0, used=0.0))
    a["n"] += 1
    a["frac"] = max(a["frac"], r["max_d_over_max_ref"])
    a["used"] = max(a["used"], r["used"])
print("| test | tensor | bound: rtol·|ref| + frac·max|ref| | checks | measured max|d|/max|ref| | largest share of the bound |")
print("|---|---|---|---|---|---|")
for (test, tensor, rtol, frac), a in rows.items():
    print(f"| `{test.split('::')[-1]}` ({test.split('::')[0].split('/')[-1]}) | {tensor} | {rtol:g} · {frac:g} | {a['n']} | "
          f"{a['frac']:.2e} | {a['used']:.2f} |")
