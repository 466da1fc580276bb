"""In-tree build of the native parts (no JIT cache: the .so files travel with
the repo snapshot to the GPU box).

  openr_amd/lib/libopenr_hip.so      hipcc, gfx950: C ABI + SPF kernels
  openr_amd/_openr_host*.so          g++: drop-in LinkState / SpfSolver host
                                     library (links libopenr_hip), pybind11
  oracle/build/openr_oracle*.so      g++: CPU oracle (test infrastructure)
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "lib")
HIP_LIB = os.path.join(LIB_DIR, "libopenr_hip.so")
EXT = sysconfig.get_config_var("EXT_SUFFIX")
HOST_MOD = os.path.join(PKG, "_openr_host" + EXT)
ARCH = os.environ.get("OPENR_HIP_ARCH", "gfx950")

HIP_SRCS = [os.path.join(CSRC, "orh_api.hip"), os.path.join(CSRC, "kernels", "spf_kernels.hip"),
            os.path.join(CSRC, "kernels", "route_kernels.hip"),
            os.path.join(CSRC, "kernels", "whatif_kernels.hip"),
            os.path.join(CSRC, "kernels", "ksp_kernels.hip")]
HOST_SRCS = [os.path.join(CSRC, "host", f) for f in ("link_state.cpp", "prefix_state.cpp", "spf_solver.cpp",
                                                   "rib_policy.cpp", "thrift_compact.cpp",
                                                   "decision_ingest.cpp", "multi_device.cpp", "whatif_batch.cpp",
                                                   "host_py.cpp")]


def _hipcc() -> str:
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: cannot build libopenr_hip for " + ARCH)


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def _includes(src, seen=None):
    """The source and every header it reaches through #include "..." lines."""
    import re
    seen = set() if seen is None else seen
    if src in seen or not os.path.exists(src):
        return seen
    seen.add(src)
    with open(src) as f:
        for m in re.finditer(r'^\s*#\s*include\s+"([^"]+)"', f.read(), re.M):
            _includes(os.path.normpath(os.path.join(os.path.dirname(src), m.group(1))), seen)
    return seen


def build_hip_lib(force: bool = False) -> str:
    """One object per HIP source (rebuilt when it or a header it includes
    changed), compiled in parallel, then one shared link."""
    obj_dir = os.path.join(LIB_DIR, "obj")
    os.makedirs(obj_dir, exist_ok=True)
    objs = [os.path.join(obj_dir, os.path.basename(s) + ".o") for s in HIP_SRCS]
    todo = [(s, o) for s, o in zip(HIP_SRCS, objs) if force or _stale(o, sorted(_includes(s)))]

    def compile_one(so):
        src, obj = so
        _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c",
              "-Wno-unused-value", "-Wno-unused-result", "-o", obj + ".tmp", src])
        os.replace(obj + ".tmp", obj)

    with ThreadPoolExecutor(max(1, len(todo))) as ex:
        list(ex.map(compile_one, todo))
    if force or todo or _stale(HIP_LIB, objs):
        tmp = HIP_LIB + ".tmp"
        _run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-o", tmp] + objs)
        os.replace(tmp, HIP_LIB)
    return HIP_LIB


def build_host_module(force: bool = False) -> str:
    """One object per host source (rebuilt when it or a header it includes
    changed), compiled in parallel, then one shared link against libopenr_hip."""
    import pybind11
    obj_dir = os.path.join(LIB_DIR, "obj")
    os.makedirs(obj_dir, exist_ok=True)
    objs = [os.path.join(obj_dir, os.path.basename(s) + ".o") for s in HOST_SRCS]
    todo = [(s, o) for s, o in zip(HOST_SRCS, objs) if force or _stale(o, sorted(_includes(s)))]

    def compile_one(so):
        src, obj = so
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-c",
              f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
              f"-I{os.path.join(ROOT, 'include')}", "-o", obj + ".tmp", src])
        os.replace(obj + ".tmp", obj)

    with ThreadPoolExecutor(max(1, min(8, len(todo)))) as ex:
        list(ex.map(compile_one, todo))
    if force or todo or _stale(HOST_MOD, objs + [HIP_LIB]):
        tmp = HOST_MOD + ".tmp"
        _run(["g++", "-shared", "-fPIC", "-o", tmp] + objs +
             [f"-L{LIB_DIR}", "-lopenr_hip", "-Wl,-rpath,$ORIGIN/lib"])
        os.replace(tmp, HOST_MOD)
    return HOST_MOD


def build_oracle() -> None:
    """CPU oracle (test infrastructure); built here so the GPU box has it."""
    _run(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


def build_all(force: bool = False) -> None:
    with ThreadPoolExecutor(2) as ex:
        f_oracle = ex.submit(build_oracle)
        build_hip_lib(force)
        build_host_module(force)
        f_oracle.result()


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    print("built", HIP_LIB, HOST_MOD)
