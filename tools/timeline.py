"""Per-step kernel timeline from a rocprofv3 kernel trace: durations and idle gaps of the last
step (delimited by k_render_bwd), plus per-step busy / wall totals."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gs::", "")[:44] for r in rows]
idx = [i for i, n in enumerate(names) if n.startswith("k_render_bwd")]
for a, b in zip(idx[:-1], idx[1:]):
    s, e = int(rows[a]["End_Timestamp"]), int(rows[b]["End_Timestamp"])
    busy = sum(int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"]) for i in range(a + 1, b + 1))
    print(f"step {(e - s) / 1e3:8.1f} us  busy {busy / 1e3:8.1f} us  kernels {b - a}")
a, b = idx[-2], idx[-1]
prev = int(rows[a]["End_Timestamp"])
for i in range(a + 1, b + 1):
    r = rows[i]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"  {names[i]:46s} {(e - s) / 1e3:8.2f} us   gap {(s - prev) / 1e3:7.2f}")
    prev = e
