"""Build the native engine in-tree.

Three explicit stages, no source translation step:
  1. csrc/kernels/*.hip -> build/kernels/*.o with hipcc, device code for gfx950
     only;
  2. csrc/engine/*.cpp (except bind.cpp) + csrc/capi/*.cpp -> build/host/*.o with
     the host C++ compiler against ATen/c10d, linked with the kernel objects into
     gpu_mapreduce_amd/libmrhip.so — the engine + native MapReduce + MR_* C API
     (what C/C++ programs link against);
  3. the Python module gpu_mapreduce_amd/_C (csrc/engine/bind.cpp), linked to
     libmrhip.so.
Steps 1-2 are parallel (MAX_JOBS) and incremental on source/header mtimes.
Usage: python setup.py build_ext --inplace
"""
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

from setuptools import setup
from torch.utils.cpp_extension import BuildExtension, CppExtension, include_paths

here = os.path.dirname(os.path.abspath(__file__))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("MRH_OFFLOAD_ARCH", "gfx950")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
CXX = os.environ.get("CXX", "g++")
PKG = os.path.join(here, "gpu_mapreduce_amd")
BUILD = os.path.join(here, "build")
LIB = os.path.join(PKG, "libmrhip.so")

hip_sources = sorted(glob.glob(os.path.join(here, "csrc", "kernels", "*.hip")))
kernel_headers = sorted(glob.glob(os.path.join(here, "csrc", "kernels", "*.h")))
host_sources = sorted(s for s in glob.glob(os.path.join(here, "csrc", "engine", "*.cpp"))
                      if not s.endswith("bind.cpp")) + sorted(glob.glob(os.path.join(here, "csrc", "capi", "*.cpp"))) + \
    sorted(s for s in glob.glob(os.path.join(here, "csrc", "oink", "*.cpp")) if not s.endswith("main.cpp"))
host_headers = sorted(glob.glob(os.path.join(here, "csrc", "engine", "*.h")) +
                      glob.glob(os.path.join(here, "csrc", "capi", "*.h")) +
                      glob.glob(os.path.join(here, "csrc", "oink", "*.h"))) + kernel_headers
OINK_MAIN = os.path.join(here, "csrc", "oink", "main.cpp")
OINK_BIN = os.path.join(PKG, "bin", "oink")
# native app programs (csrc/apps/*.cpp -> gpu_mapreduce_amd/bin/<name>)
APP_SOURCES = sorted(glob.glob(os.path.join(here, "csrc", "apps", "*.cpp")))
APP_HEADERS = sorted(glob.glob(os.path.join(here, "csrc", "apps", "*.h")))

HIPFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
            "-Wno-unused-result", "-Wno-unused-value", "-I", os.path.join(here, "csrc")]


def _torch_lib():
    import torch
    return os.path.join(os.path.dirname(torch.__file__), "lib")


def _abi():
    import torch
    return int(torch._C._GLIBCXX_USE_CXX11_ABI)


HOSTDEFS = ["-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={_abi()}"]
HOSTFLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wno-unused-result", "-Wno-sign-compare", *HOSTDEFS,
             "-I", os.path.join(here, "csrc"), "-I", os.path.join(ROCM, "include")] + \
            [f"-I{p}" for p in include_paths()]
LINKLIBS = [f"-L{os.path.join(ROCM, 'lib')}", f"-L{_torch_lib()}", "-lamdhip64", "-lhiprtc", "-lc10_hip", "-ltorch_hip",
            "-lc10", "-ltorch", "-ltorch_cpu", "-lrocprofiler-sdk-roctx",
            # RCCL: no -lrccl on purpose. The nccl* symbols resolve at load
            # time from the librccl that libtorch_hip already depends on, so a
            # process never maps two RCCL copies (torch ships its own; a
            # NEEDED librccl.so.1 would pull /opt/rocm's in beside it)
            f"-Wl,-rpath,{_torch_lib()}", f"-Wl,-rpath,{os.path.join(ROCM, 'lib')}"]


def _stale(obj, deps):
    return not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(d) for d in deps)


def _compile_all(jobs):
    os.makedirs(os.path.join(BUILD, "kernels"), exist_ok=True)
    os.makedirs(os.path.join(BUILD, "host"), exist_ok=True)
    tasks = []
    for s in hip_sources:
        o = os.path.join(BUILD, "kernels", os.path.splitext(os.path.basename(s))[0] + ".o")
        tasks.append((o, [HIPCC, *HIPFLAGS, "-c", s, "-o", o], [s] + kernel_headers))
    for s in host_sources:
        sub = os.path.basename(os.path.dirname(s))
        o = os.path.join(BUILD, "host", sub + "_" + os.path.splitext(os.path.basename(s))[0] + ".o")
        tasks.append((o, [CXX, *HOSTFLAGS, "-c", s, "-o", o], [s] + host_headers))

    def one(t):
        o, cmd, deps = t
        if _stale(o, deps):
            print(" ".join(cmd), flush=True)
            subprocess.run(cmd, check=True)
        return o
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        return list(ex.map(one, tasks))


def build_native():
    objs = _compile_all(int(os.environ.get("MAX_JOBS", "8")))
    if _stale(LIB, objs):
        cmd = [CXX, "-shared", "-o", LIB, *objs, *LINKLIBS]
        print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    # the oink executable (reference oink/main.cpp), linked to libmrhip.so
    if _stale(OINK_BIN, [OINK_MAIN, LIB] + host_headers):
        os.makedirs(os.path.dirname(OINK_BIN), exist_ok=True)
        cmd = [CXX, *HOSTFLAGS, OINK_MAIN, "-o", OINK_BIN, f"-L{PKG}", "-lmrhip", "-Wl,-rpath,$ORIGIN/..", *LINKLIBS]
        print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    def app(src):
        exe = os.path.join(PKG, "bin", os.path.splitext(os.path.basename(src))[0])
        if _stale(exe, [src, LIB] + host_headers + APP_HEADERS):
            cmd = [CXX, *HOSTFLAGS, src, "-o", exe, f"-L{PKG}", "-lmrhip", "-Wl,-rpath,$ORIGIN/..", *LINKLIBS]
            print(" ".join(cmd), flush=True)
            subprocess.run(cmd, check=True)
    os.makedirs(os.path.join(PKG, "bin"), exist_ok=True)
    with ThreadPoolExecutor(max_workers=max(1, int(os.environ.get("MAX_JOBS", "8")))) as ex:
        list(ex.map(app, APP_SOURCES))
    return LIB


class Build(BuildExtension):
    def build_extensions(self):
        build_native()
        super().build_extensions()


setup(
    name="gpu_mapreduce_amd",
    version="0.1.0",
    packages=["gpu_mapreduce_amd"],
    ext_modules=[
        CppExtension(
            "gpu_mapreduce_amd._C",
            [os.path.join("csrc", "engine", "bind.cpp")],
            include_dirs=[os.path.join(here, "csrc"), os.path.join(ROCM, "include")],
            define_macros=[("__HIP_PLATFORM_AMD__", "1"), ("USE_ROCM", "1")],
            library_dirs=[PKG, os.path.join(ROCM, "lib"), _torch_lib()],
            libraries=["mrhip", "amdhip64", "c10_hip", "torch_hip"],
            extra_compile_args=["-O3", "-std=c++17", "-Wno-unused-result", "-Wno-sign-compare"],
            extra_link_args=["-Wl,-rpath,$ORIGIN", f"-Wl,-rpath,{os.path.join(ROCM, 'lib')}"],
        )
    ],
    cmdclass={"build_ext": Build.with_options(use_ninja=True)},
)
