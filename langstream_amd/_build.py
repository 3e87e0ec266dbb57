"""In-tree native build for langstream_amd.

Two shared objects are produced next to the sources (so they travel with the
repo snapshot to the GPU box):

* ``langstream_amd/ops/_hip_ops.so`` -- the HIP/CDNA4 kernels (``ops/csrc/*.hip``),
  compiled with ``hipcc --offload-arch=gfx950`` and linked against libtorch so
  the kernels take ``at::Tensor`` arguments and launch on the current HIP
  stream (graph-capturable).
* ``langstream_amd/native/_lsnative.so`` -- host-side C++ runtime pieces
  (BPE/WordPiece tokenizer, in-memory partitioned topic log, paged-KV block
  allocator), compiled with g++ and bound with pybind11.  No torch dependency.

The build is incremental: an object is rebuilt when its source (or any header
in the same directory) is newer than the object.  Compilation runs in a small
process pool (the container has 8 CPUs; the GPU box exports MAX_JOBS=16).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shlex
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
OPS_DIR = os.path.join(ROOT, "ops")
CSRC = os.path.join(OPS_DIR, "csrc")
NATIVE_DIR = os.path.join(ROOT, "native")
BUILD_DIR = os.path.join(ROOT, "_objs")
HIP_SO = os.path.join(OPS_DIR, "_hip_ops.so")
NATIVE_SO = os.path.join(NATIVE_DIR, "_lsnative.so")
ARCH = os.environ.get("LANGSTREAM_GPU_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _jobs() -> int:
    try:
        return max(1, min(int(os.environ.get("MAX_JOBS", "8")), 16))
    except ValueError:
        return 8


def _newest(paths) -> float:
    m = 0.0
    for p in paths:
        try:
            m = max(m, os.path.getmtime(p))
        except OSError:
            pass
    return m


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(shlex.quote(c) for c in cmd) + "\n" + r.stdout)


def _torch_flags():
    import torch
    from torch.utils import cpp_extension as ce

    inc = []
    for p in ce.include_paths(device_type="cuda"):
        inc += ["-I", p]
    inc += ["-I", sysconfig.get_paths()["include"]]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    defs = [
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-DTORCH_EXTENSION_NAME=_hip_ops",
        "-DUSE_ROCM=1",
    ]
    torch_lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    libs = [
        "-L", torch_lib,
        f"-Wl,-rpath,{torch_lib}",
        "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip",
        "-lamdhip64",
    ]
    return inc, defs, libs


def build_hip(verbose: bool = False) -> str:
    """Compile every ``ops/csrc/*.hip`` for gfx950 and link ``_hip_ops.so``."""
    os.makedirs(BUILD_DIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    headers = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "*.cuh"))
    hdr_time = _newest(headers)
    inc, defs, libs = _torch_flags()
    cflags = [
        f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=fast",
        "-Wno-unused-result", "-Wno-deprecated-declarations", "-Wno-unused-command-line-argument",
        "-fgpu-rdc" if False else "-fno-gpu-rdc",
    ]
    jobs = []
    objs = []
    for s in srcs:
        o = os.path.join(BUILD_DIR, os.path.basename(s) + ".o")
        objs.append(o)
        if not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(s), hdr_time):
            jobs.append([HIPCC, *cflags, *defs, *inc, "-I", CSRC, "-c", s, "-o", o])
    if jobs:
        with cf.ThreadPoolExecutor(_jobs()) as ex:
            list(ex.map(_run, jobs))
    if jobs or not os.path.exists(HIP_SO) or os.path.getmtime(HIP_SO) < _newest(objs):
        tmp = HIP_SO + ".tmp"
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, *libs, "-o", tmp])
        os.replace(tmp, HIP_SO)
    if verbose:
        print(f"[build] {HIP_SO} ({len(jobs)} objects rebuilt)")
    return HIP_SO


def build_native(verbose: bool = False) -> str:
    """Compile the host C++ runtime (``native/*.cpp``) into ``_lsnative.so``."""
    import pybind11

    os.makedirs(BUILD_DIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(NATIVE_DIR, "*.cpp")))
    headers = glob.glob(os.path.join(NATIVE_DIR, "*.h"))
    hdr_time = _newest(headers)
    inc = ["-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"], "-I", NATIVE_DIR]
    cflags = ["-O3", "-fPIC", "-std=c++17", "-fvisibility=hidden", "-pthread", "-Wall", "-Wno-sign-compare"]
    jobs, objs = [], []
    for s in srcs:
        o = os.path.join(BUILD_DIR, "native_" + os.path.basename(s) + ".o")
        objs.append(o)
        if not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(s), hdr_time):
            jobs.append(["g++", *cflags, *inc, "-c", s, "-o", o])
    if jobs:
        with cf.ThreadPoolExecutor(_jobs()) as ex:
            list(ex.map(_run, jobs))
    if jobs or not os.path.exists(NATIVE_SO) or os.path.getmtime(NATIVE_SO) < _newest(objs):
        tmp = NATIVE_SO + ".tmp"
        _run(["g++", "-shared", "-fPIC", "-pthread", *objs, "-o", tmp])
        os.replace(tmp, NATIVE_SO)
    if verbose:
        print(f"[build] {NATIVE_SO} ({len(jobs)} objects rebuilt)")
    return NATIVE_SO


def build_all(verbose: bool = True) -> None:
    build_native(verbose)
    build_hip(verbose)


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which in ("all", "native"):
        build_native(True)
    if which in ("all", "hip"):
        build_hip(True)
