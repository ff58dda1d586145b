"""Builds diff_gaussian_rasterization/_gs_ext*.so, the torch C++ host fast path of the ctypes bridge
(csrc/gs_torch_ext.cpp), in place:  python setup_ext.py build_ext --inplace
(__graft_entry__.build() runs it; the extension resolves libgsrast.so's C ABI at run time)."""
import os
import tempfile

from setuptools import setup
from torch.utils.cpp_extension import BuildExtension, CppExtension

HERE = os.path.dirname(os.path.abspath(__file__))
os.chdir(HERE)
setup(
    name="gs_torch_ext",
    ext_modules=[CppExtension("diff_gaussian_rasterization._gs_ext", ["csrc/gs_torch_ext.cpp"],
                              include_dirs=["/opt/rocm/include", os.path.join(HERE, "..", "include")],
                              extra_compile_args=["-O2", "-g0", "-D__HIP_PLATFORM_AMD__=1"],
                              extra_link_args=["-s"])],
    cmdclass={"build_ext": BuildExtension},
    # objects in a temporary directory; the module lands in diff_gaussian_rasterization/
    script_args=["build_ext", "--inplace", "-t", os.path.join(tempfile.gettempdir(), "gs_ext_build"),
                 "-b", os.path.join(tempfile.gettempdir(), "gs_ext_lib")],
)
