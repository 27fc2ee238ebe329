"""Build the native engine in-tree: gpu_mapreduce_amd/_C*.so

Two explicit stages, no source translation step:
  1. csrc/kernels/*.hip -> build/kernels/*.o with hipcc, device code for gfx950
     only (parallel, incremental on source/header mtimes);
  2. csrc/engine/*.cpp (ATen / c10d / pybind11 host code) with the host C++
     compiler, linked with the kernel objects, libamdhip64 and torch's HIP libs.
Usage: python setup.py build_ext --inplace   (MAX_JOBS bounds hipcc parallelism)
"""
import glob
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

from setuptools import setup
from torch.utils.cpp_extension import BuildExtension, CppExtension

here = os.path.dirname(os.path.abspath(__file__))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("MRH_OFFLOAD_ARCH", "gfx950")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
KDIR = os.path.join("csrc", "kernels")
OBJDIR = os.path.join(here, "build", "kernels")
hip_sources = sorted(glob.glob(os.path.join(KDIR, "*.hip")))
kernel_headers = sorted(glob.glob(os.path.join(KDIR, "*.h")))
cpp_sources = sorted(glob.glob(os.path.join("csrc", "engine", "*.cpp")))
HIPFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
            "-Wno-unused-result", "-Wno-unused-value", "-I", os.path.join(here, "csrc")]


def _obj(src):
    return os.path.join(OBJDIR, os.path.splitext(os.path.basename(src))[0] + ".o")


def compile_kernels():
    os.makedirs(OBJDIR, exist_ok=True)
    hdr_t = max([os.path.getmtime(h) for h in kernel_headers] + [0])

    def one(src):
        o = _obj(src)
        if os.path.exists(o) and os.path.getmtime(o) >= max(os.path.getmtime(src), hdr_t):
            return o
        cmd = [HIPCC, *HIPFLAGS, "-c", src, "-o", o]
        print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        return o
    jobs = int(os.environ.get("MAX_JOBS", "8"))
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        return list(ex.map(one, hip_sources))


class Build(BuildExtension):
    def build_extensions(self):
        objs = compile_kernels()
        for ext in self.extensions:
            ext.extra_objects = list(objs)
        super().build_extensions()


def _torch_lib():
    import torch
    return os.path.join(os.path.dirname(torch.__file__), "lib")


setup(
    name="gpu_mapreduce_amd",
    version="0.1.0",
    packages=["gpu_mapreduce_amd"],
    ext_modules=[
        CppExtension(
            "gpu_mapreduce_amd._C",
            cpp_sources,
            include_dirs=[os.path.join(here, "csrc"), os.path.join(ROCM, "include")],
            define_macros=[("__HIP_PLATFORM_AMD__", "1"), ("USE_ROCM", "1")],
            library_dirs=[os.path.join(ROCM, "lib"), _torch_lib()],
            libraries=["amdhip64", "c10_hip", "torch_hip"],
            extra_compile_args=["-O3", "-std=c++17", "-Wno-unused-result", "-Wno-sign-compare"],
            extra_link_args=[f"-Wl,-rpath,{os.path.join(ROCM, 'lib')}"],
        )
    ],
    cmdclass={"build_ext": Build.with_options(use_ninja=True)},
)
