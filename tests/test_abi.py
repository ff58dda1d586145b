"""The C-ABI library loads here (no GPU needed) and exports every symbol include/gsrast.h declares;
the Python binding declares every one of them; the code object targets gfx950."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "gsrast.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gs_[a-z0-9_]+)\s*\(", txt)) - {"gs_alloc_fn"})


def test_library_exports_every_header_symbol():
    from diff_gaussian_rasterization import _native

    lib = _native.load()
    syms = _header_symbols()
    assert len(syms) >= 18
    for s in syms:
        assert hasattr(lib, s), f"libgsrast.so does not export {s}"
    assert set(syms) == set(_native.SIGNATURES), set(syms) ^ set(_native.SIGNATURES)
    want = int(re.search(r"#define GSRAST_ABI_VERSION (\d+)", open(os.path.join(ROOT, "include", "gsrast.h")).read()).group(1))
    assert want == 17 and lib.gs_abi_version() == want


def test_graft_build_checks_the_header_abi():
    """__graft_entry__.build() compares the loaded library's ABI with include/gsrast.h (not a literal)."""
    src = open(os.path.join(ROOT, "__graft_entry__.py")).read()
    assert "GSRAST_ABI_VERSION" in src and "gs_abi_version() ==" not in src


def test_sizing_functions_run_without_gpu():
    from diff_gaussian_rasterization import _native

    lib = _native.load()
    assert lib.gs_geom_buffer_bytes(1_000_000) > 60 * 1_000_000
    assert lib.gs_binning_buffer_bytes(3_000_000, 1920, 1080) > 20 * 3_000_000
    assert lib.gs_image_buffer_bytes(1920, 1080) >= 8 * 1920 * 1080
    assert lib.gs_grad_buffer_bytes(10) >= 360


def test_binning_layout_count_recovers_the_sized_layout():
    """The backward recovers the binning buffer's layout count from its byte size
    (gs_binning_layout_count): the largest count whose gs_binning_buffer_bytes fits.  That is only the
    layout the buffer was sized for if the size never decreases with the count -- in particular
    across the radix sort's block-count steps, where sort_plan's block count drops (every
    4096 x 2048 = 2^23 instances).  Counts around those steps and random ones."""
    import random

    from diff_gaussian_rasterization import _native

    lib = _native.load()
    W, H = 1920, 1080
    step = 1 << 23
    counts = [1, 63, 64, 65, 2047, 2048, 2049, 4_330_000]
    for k in (1, 2, 3):
        counts += [k * step + d for d in (-2049, -2048, -1, 0, 1, 2048, 2049)]
    rng = random.Random(0)
    counts += [rng.randrange(1, 40_000_000) for _ in range(40)]
    for c in sorted(counts):
        b = lib.gs_binning_buffer_bytes(c, W, H)
        assert lib.gs_binning_buffer_bytes(c + 1, W, H) >= b, c
        assert lib.gs_binning_buffer_bytes(c + 2048, W, H) >= b, c
        L = lib.gs_binning_layout_count(b, W, H)
        assert L >= c and lib.gs_binning_buffer_bytes(L, W, H) == b, (c, L)


def test_code_object_targets_gfx950():
    from diff_gaussian_rasterization import _native

    data = open(_native.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_knn_and_validation_errors_without_gpu():
    """Argument validation happens before any device work: errors are reported, not crashes."""
    import ctypes

    from diff_gaussian_rasterization import _native

    lib = _native.load()
    nr = ctypes.c_longlong(7)
    rc = lib.gs_forward_preprocess(4, 0, 1, None, 16, 16, None, None, None, None, None, 1.0, None, None, None,
                                   None, None, 0.5, 0.5, 0, None, None, ctypes.byref(nr), 0, None)
    assert rc != 0 and "missing" in _native.last_error()
    rc = lib.gs_forward_preprocess(0, 0, 1, None, 0, 16, None, None, None, None, None, 1.0, None, None, None,
                                   None, None, 0.5, 0.5, 0, None, None, ctypes.byref(nr), 0, None)
    assert rc != 0 and "image size" in _native.last_error()


def test_numerics_mode_default_and_env():
    """Fast exp2 is the default; GSRAST_EXACT_EXP=1 selects the bit-exact mode (fresh processes)."""
    import subprocess
    import sys

    code = ("import sys; sys.path.insert(0, %r); from diff_gaussian_rasterization import _native; "
            "L = _native.load(); print(L.gs_set_exact_exp(0), L.gs_set_exact_exp(1))") % os.path.join(
                ROOT, "gaussian-splatting-skysphere_amd")
    env = {k: v for k, v in os.environ.items() if k != "GSRAST_EXACT_EXP"}
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
    assert out.stdout.split() == ["0", "0"]
    env["GSRAST_EXACT_EXP"] = "1"
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
    assert out.stdout.split() == ["1", "0"]


def test_geom_flags_offset_lies_in_the_counters():
    """gs_geom_flags_offset (ABI 17): a 4-aligned word inside the geometry buffer, in its 64-B
    counters block (CNT_ERR = word 2), for every P."""
    from diff_gaussian_rasterization import _native

    lib = _native.load()
    for P in (0, 1, 255, 256, 3000, 1_000_000, 5_000_000):
        off = lib.gs_geom_flags_offset(P)
        assert off % 4 == 0 and off + 4 <= lib.gs_geom_buffer_bytes(P), P
        assert (off - 8) % 256 == 0, P  # the counters block is 256-B aligned, the flags are its word 2


def test_row_waits_validation_on_the_host():
    """gs_set_row_waits (ABI 17) checks its chunk bounds on the host (no GPU call): from row 0,
    increasing, at most 64 chunks; n = 0 clears; null events are allowed (nothing to wait for)."""
    import ctypes

    from diff_gaussian_rasterization import _native

    lib = _native.load()

    def set_(bounds):
        n = len(bounds) - 1
        b = (ctypes.c_int * len(bounds))(*bounds)
        e = (ctypes.c_void_p * max(n, 1))()
        return lib.gs_set_row_waits(n, ctypes.cast(b, ctypes.c_void_p), ctypes.cast(e, ctypes.c_void_p))

    assert set_([0, 100, 4096]) == 0
    assert lib.gs_set_row_waits(0, None, None) == 0
    assert set_([1, 100]) != 0 and b"row 0" in lib.gs_last_error()
    assert set_([0, 100, 100]) != 0 and b"increase" in lib.gs_last_error()
    assert set_(list(range(0, 66 * 10, 10))) != 0  # 65 chunks
    assert lib.gs_set_row_waits(-1, None, None) != 0
    assert lib.gs_set_row_waits(0, None, None) == 0


def test_row_chunks_follow_the_preprocess_launch_rule():
    """gs_train.row_chunks (the activation's chunks) uses the rasterizer's rule
    (csrc/gs_forward.hip launch_row_chunks): 256-row blocks, a block in the chunk that holds its last
    row; the chunks are contiguous, cover [0, P), and keep every event in order."""
    import gs_train

    evs = [object() for _ in range(4)]
    for P in (1, 255, 256, 700, 1000, 5000, 100_000):
        for cuts in ([0, P], [0, P // 3, 2 * P // 3, P], [0, 1, 2, P], [0, 256, 512, 768, P]):
            cuts = sorted(set(min(max(c, 0), P) for c in cuts))
            if len(cuts) < 2 or cuts[0] != 0 or cuts[-1] != P:
                continue
            waits = [(cuts[k], cuts[k + 1], evs[k % 4]) for k in range(len(cuts) - 1)]
            out = gs_train.row_chunks(P, waits)
            assert out[0][0] == 0 and out[-1][1] == P
            assert all(out[k][1] == out[k + 1][0] for k in range(len(out) - 1))
            assert all(lo % 256 == 0 for lo, _, _ in out)
            # the block holding row r launches in a chunk whose waits include the chunk of r
            seen = [e for _, _, e in out if e is not None]
            assert seen == [e for _, _, e in waits][:len(seen)]
            for lo, hi, _ in out:
                for r in (lo, hi - 1):
                    if lo < hi:
                        last_row = min(256 * (r // 256) + 255, P - 1)
                        k_needed = next(k for k, (a, b, _) in enumerate(waits) if a <= last_row < b)
                        k_have = sum(1 for lo2, _, e in out if e is not None and lo2 <= lo)
                        assert k_have >= k_needed + 1 or (k_needed == len(waits) - 1 and k_have == len(seen)), (P, cuts)
