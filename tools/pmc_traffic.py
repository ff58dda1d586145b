"""HBM traffic per launch from rocprofv3 --pmc passes (gpurun_out/pmc_fetch, pmc_write).

traffic = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md §HBM (FETCH_SIZE reports half of a wide streaming read).
Writes {workload: {kernel: bytes_per_launch}} to profiles/pmc_traffic.json (merged), keyed by the
profile names bench.py uses (k_render_bwd -> render_bwd)."""
import csv
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
workload = sys.argv[2] if len(sys.argv) > 2 else "c3"
out_path = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                              "pmc_traffic.json")


def per_kernel(counter, d):
    acc = defaultdict(list)
    f = os.path.join(root, d, "run_counter_collection.csv")
    if not os.path.exists(f):
        return {}
    per_dispatch = defaultdict(float)
    names = {}
    for row in csv.DictReader(open(f)):
        if row["Counter_Name"] != counter:
            continue
        k = row["Kernel_Name"]
        if "gs::" not in k:
            continue
        short = k.split("(")[0].replace("void ", "").split("<")[0].replace("gs::", "")
        short = short[2:] if short.startswith("k_") else short
        short = {"duplicate_lb": "duplicate", "preprocess_bwd_reg": "preprocess_bwd", "render_fwd_q": "render_fwd",
                 "render_bwd_tw": "render_bwd"}.get(short, short)  # bench.py names
        per_dispatch[row["Dispatch_Id"]] += float(row["Counter_Value"])
        names[row["Dispatch_Id"]] = short
    for disp, v in per_dispatch.items():
        acc[names[disp]].append(v)
    return {k: sum(v) / len(v) for k, v in acc.items()}


fetch = per_kernel("FETCH_SIZE", "pmc_fetch")
write = per_kernel("WRITE_SIZE", "pmc_write")
valu = per_kernel("SQ_INSTS_VALU", "pmc_sq2")
if valu:  # wave-level VALU instructions per launch (device total), for the compute roofline
    vpath = os.path.join(os.path.dirname(out_path), "pmc_valu.json")
    vdata = json.load(open(vpath)) if os.path.exists(vpath) else {}
    vdata[workload] = {k: int(round(v)) for k, v in sorted(valu.items())}
    json.dump(vdata, open(vpath, "w"), indent=1, sort_keys=True)
res = {}
for k in sorted(set(fetch) & set(write)):
    res[k] = int(round((2 * fetch[k] + write[k]) * 1024))
    print(f"{k:18s} fetch(x2) {2 * fetch[k] * 1024 / 1e6:9.1f} MB  write {write[k] * 1024 / 1e6:9.1f} MB  "
          f"traffic {res[k] / 1e6:9.1f} MB")
data = json.load(open(out_path)) if os.path.exists(out_path) else {}
data[workload] = res
json.dump(data, open(out_path, "w"), indent=1, sort_keys=True)
