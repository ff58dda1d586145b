"""Measured parity errors of the GPU tests (DESIGN.md §0 / §2 contract table).

With GS_PARITY_REPORT=<path> set, every tolerance check of tests/test_gpu_parity.py and
tests/test_gpu_dense.py appends one JSON line: the test, the tensor, the bound it asserts
(|d| <= rtol |ref| + frac max|ref|), the measured max|d| / max|ref| and the largest fraction of the
bound used anywhere (`used` <= 1 passes).  tools/parity_table.py reduces the file to the table."""
import json
import os

import numpy as np


def record(name, gpu, ref, rtol, frac, keep=None):
    path = os.environ.get("GS_PARITY_REPORT")
    if not path:
        return
    gpu = np.asarray(gpu, np.float64)
    ref = np.asarray(ref, np.float64)
    if keep is not None:
        gpu, ref = gpu[keep], ref[keep]
    if ref.size == 0:
        return
    scale = float(np.abs(ref).max())
    d = np.abs(gpu - ref)
    tol = rtol * np.abs(ref) + frac * scale
    used = float((d / np.maximum(tol, 1e-300)).max()) if scale > 0 else 0.0
    test = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    with open(path, "a") as f:
        f.write(json.dumps({"test": test, "tensor": name, "rtol": rtol, "frac": frac,
                            "max_d_over_max_ref": float(d.max()) / scale if scale > 0 else 0.0,
                            "used": used}) + "\n")
