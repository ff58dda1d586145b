"""Aggregate rocprofv3 --pmc counter_collection CSVs per kernel (mean per dispatch)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
agg = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
pat = sys.argv[2] if len(sys.argv) > 2 else "pmc_"
for f in sorted(glob.glob(os.path.join(root, pat + "*", "run_counter_collection.csv"))):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        short = k.split("(")[0].replace("void ", "").split("<")[0].replace("gs::", "")
        if "at::native" in k:
            continue
        key = (short, row["Dispatch_Id"], os.path.basename(os.path.dirname(f)))
        agg[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
        dur[short].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
for kname, cs in agg.items():
    vals = {c: sum(v) / len(v) for c, v in cs.items()}
    print(kname)
    for c in sorted(vals):
        print(f"   {c:28s} {vals[c]:.4g}")
