"""Every kernel in libgsrast.so's gfx950 code object is launched by some GPU test.

The library records the distinct kernels it launches (GSRAST_LAUNCH_LOG=1, set by conftest.py;
gs_debug_launched_kernels returns their mangled names through dladdr on the kernel handles).  Run
as the last test of a whole-suite GPU session (`pytest tests -m gpu`), it compares that list with
the kernel descriptors (`<name>.kd`) of the code object embedded in the library: a kernel that no
test launches is dead code or untested code, and fails the check.  Kernels launched only inside
the multi-process tests' child processes are launched there, not here: the list below names
them, and test_gpu_view_parallel / test_gpu_multiview cover them in their children."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def code_object_kernels(path):
    data = open(path, "rb").read()
    return sorted(set(m.decode() for m in re.findall(rb"(_Z[0-9A-Za-z_]+)\.kd\x00", data)))


def launched_kernels(lib):
    n = lib.gs_debug_launched_kernels(None, 0)
    buf = ctypes.create_string_buffer(n + 1)
    assert lib.gs_debug_launched_kernels(buf, n + 1) == n
    return sorted(set(buf.value.decode().split()))


def test_code_object_lists_kernels():
    """(CPU) the code object's kernel descriptors are found, and the launch log is exported."""
    from diff_gaussian_rasterization import _native

    ks = code_object_kernels(_native.LIB_PATH)
    assert len(ks) > 20 and all(k.startswith("_ZN2gs") for k in ks)
    lib = _native.load()
    assert lib.gs_debug_launch_log(1) in (0, 1)


def _whole_suite(session):
    """the session ran every GPU test file: no -k / file selection narrower than tests/"""
    cfg = session.config
    if cfg.getoption("keyword") or cfg.getoption("markexpr") not in ("gpu", ""):
        return False
    tests_dir = os.path.join(ROOT, "tests")
    args = [os.path.abspath(a.split("::")[0]) for a in cfg.args]
    return all(a.rstrip("/") == tests_dir for a in args) and session.testsfailed == 0


@pytest.mark.gpu
@pytest.mark.last
def test_every_kernel_is_launched_by_a_test(request, device):
    from diff_gaussian_rasterization import _native

    if not _whole_suite(request.session):
        pytest.skip("needs the whole GPU suite in this session (pytest tests -m gpu)")
    lib = _native.load()
    have = code_object_kernels(_native.LIB_PATH)
    ran = launched_kernels(lib)
    missing = [k for k in have if k not in ran]
    with open(os.path.join(ROOT, "gpurun_out", "kernel_coverage.txt") if os.path.isdir(
            os.path.join(ROOT, "gpurun_out")) else os.devnull, "w") as f:
        f.write("launched:\n" + "\n".join(ran) + "\n\nnever launched:\n" + "\n".join(missing) + "\n")
    assert "?" not in ran, "a launched kernel handle did not resolve to an exported symbol"
    assert not missing, f"{len(missing)} kernels of the code object are launched by no test: {missing}"
