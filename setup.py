"""Build the native engine in-tree: gpu_mapreduce_amd/_C*.so

HIP kernels (csrc/kernels/*.hip) are compiled by hipcc for gfx950 only;
the engine/bindings (csrc/engine/*.cpp) by the host compiler against ATen/c10d.
Usage: PYTORCH_ROCM_ARCH=gfx950 python setup.py build_ext --inplace
"""
import glob
import os

from setuptools import setup
from torch.utils.cpp_extension import BuildExtension, CUDAExtension

os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")
here = os.path.dirname(os.path.abspath(__file__))
hip_sources = sorted(glob.glob(os.path.join("csrc", "kernels", "*.hip")))
cpp_sources = sorted(glob.glob(os.path.join("csrc", "engine", "*.cpp")))

setup(
    name="gpu_mapreduce_amd",
    version="0.1.0",
    packages=["gpu_mapreduce_amd"],
    ext_modules=[
        CUDAExtension(
            "gpu_mapreduce_amd._C",
            cpp_sources + hip_sources,
            include_dirs=[os.path.join(here, "csrc")],
            extra_compile_args={
                "cxx": ["-O3", "-std=c++17", "-Wno-unused-result", "-Wno-sign-compare"],
                "nvcc": ["-O3", "-std=c++17", "--offload-arch=gfx950", "-Wno-unused-result",
                         "-Wno-unused-value", "-munsafe-fp-atomics"],
            },
        )
    ],
    cmdclass={"build_ext": BuildExtension.with_options(use_ninja=True)},
)
