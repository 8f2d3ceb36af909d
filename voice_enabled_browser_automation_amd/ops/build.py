"""Native build driver (no setuptools/hipify involved).

* ``_vwa_kernels.so`` -- the gfx950 HIP kernel library + torch bindings. Every ``csrc/kernels/*.hip``
  is compiled with ``hipcc --offload-arch=gfx950`` into its own object (parallel, incremental),
  ``csrc/bindings.cpp`` is compiled against the torch headers, and the lot is linked against
  torch's own HIP runtime (same ``libamdhip64.so.7`` soname, so one HIP runtime per process).
* ``_vwa_native.so`` -- the CPU runtime library (grammar engine, KV block manager): plain C++17
  with pybind11, built with g++.

Both land in-tree next to this file so they travel with the repo snapshot to the GPU box.
Run: ``python -m voice_enabled_browser_automation_amd.ops.build [--force]``.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(REPO, "csrc")
BUILD = os.path.join(REPO, "build", "native")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

KERNEL_SO = os.path.join(HERE, "_vwa_kernels.so")
NATIVE_SO = os.path.join(HERE, "_vwa_native.so")


def _torch_paths():
    import torch

    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, "include"), os.path.join(root, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(root, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _py_include():
    return sysconfig.get_paths()["include"]


def _pybind_include():
    import pybind11

    return pybind11.get_include()


def _newer(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout)
        raise RuntimeError("build step failed: " + " ".join(cmd[:6]) + " ...")


def build_kernels(force: bool = False, jobs: int = 8) -> str:
    os.makedirs(BUILD, exist_ok=True)
    inc, lib, abi = _torch_paths()
    headers = glob.glob(os.path.join(CSRC, "kernels", "*.h"))
    kern_src = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    common = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result",
              "-I", os.path.join(CSRC)] + os.environ.get("VWA_HIPCC_EXTRA", "").split()  # (utils/env.py Settings documents it; build.py stays import-light)  # (experiments)
    jobs_list = []
    objs = []
    for src in kern_src:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or not _newer(obj, [src] + headers):
            jobs_list.append(common + ["-c", src, "-o", obj])
    bind_src = os.path.join(CSRC, "bindings.cpp")
    bind_obj = os.path.join(BUILD, "bindings.o")
    objs.append(bind_obj)
    if force or not _newer(bind_obj, [bind_src] + headers):
        cmd = common + ["-c", bind_src, "-o", bind_obj, f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
                        "-DTORCH_EXTENSION_NAME=_vwa_kernels", "-DUSE_ROCM=1", "-I", _py_include()]
        for i in inc:
            cmd += ["-I", i]
        jobs_list.append(cmd)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(_run, jobs_list))
    if force or jobs_list or not _newer(KERNEL_SO, objs):
        link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", KERNEL_SO] + objs + [
            "-L", lib, "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10", "-lc10_hip", "-ltorch_hip",
            f"-Wl,-rpath,{lib}"]
        _run(link)
    return KERNEL_SO


def build_native(force: bool = False) -> str:
    """CPU runtime library (grammar engine + block manager) -- g++ / pybind11."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    hdrs = glob.glob(os.path.join(CSRC, "runtime", "*.h"))
    if not srcs:
        return ""
    if not force and _newer(NATIVE_SO, srcs + hdrs):
        return NATIVE_SO
    ext = sysconfig.get_config_var("EXT_SUFFIX")  # noqa: F841 (plain .so name is importable)
    cmd = ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-I", _py_include(),
           "-I", _pybind_include(), "-I", os.path.join(CSRC, "runtime"), "-o", NATIVE_SO] + srcs
    _run(cmd)
    return NATIVE_SO


def build_all(force: bool = False) -> list[str]:
    out = []
    n = build_native(force)
    if n:
        out.append(n)
    out.append(build_kernels(force))
    return out


if __name__ == "__main__":
    print(build_all(force="--force" in sys.argv))
