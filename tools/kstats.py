"""Per-iteration kernel time table from a rocprofv3 --kernel-trace --stats output directory."""
import csv
import glob
import sys

d, steps = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1
f = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = 0.0
for r in rows:
    n = r["Name"].split("(")[0].replace("void ", "")[:40]
    per = float(r["TotalDurationNs"]) / 1e3 / steps
    tot += per
    print(f"{n:40s} calls/it {int(r['Calls']) / steps:6.2f} us/it {per:8.2f} avg {float(r['AverageNs']) / 1e3:8.2f}")
print(f"{'sum':40s} {'':16s} us/it {tot:8.2f}   ({f})")
