"""In-tree native build for kvedge_amd (gfx950 only).

Builds, with hipcc and no hipify step:
  * ``kvedge_amd/_C.so``  -- every HIP kernel in ``csrc/kernels`` plus the
    TORCH_LIBRARY bindings in ``csrc/bindings`` (loaded via torch.ops.load_library);
  * ``kvedge_amd/bin/kv_rccl_bench`` -- native RCCL all-reduce/broadcast bandwidth
    bench;
  * ``kvedge_amd/bin/kv_runtime_selftest`` -- host self-test of the native runtime.

The .so links against the HIP runtime that torch already loaded (same soname
``libamdhip64.so.7``), so there is exactly one HIP runtime per process.

Usage: ``python -m kvedge_amd._build [--force] [-j N]``.
Incremental: an object is rebuilt only when its source or any header is newer.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kvedge_amd")
CSRC = os.path.join(ROOT, "csrc")
OBJ = os.path.join(ROOT, "build", "obj")
BIN = os.path.join(PKG, "bin")
ARCH = "gfx950"
SO_PATH = os.path.join(PKG, "_C.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def hipcc() -> str:
    cand = os.path.join(ROCM, "bin", "hipcc")
    return cand if os.path.exists(cand) else (shutil.which("hipcc") or "hipcc")


def _torch_paths():
    import torch  # noqa: F401  (import only to locate headers/libs)
    from torch.utils import cpp_extension

    inc = cpp_extension.include_paths()
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _headers():
    return glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)


def _incs(src: str):
    """``#include "*.inc"`` files of a source (shared kernel bodies split over several
    translation units, e.g. conv_glds_kernel.inc): dependencies of that source only."""
    d = os.path.dirname(src)
    out = []
    with open(src) as f:
        for line in f:
            if line.startswith('#include "') and line.rstrip().endswith('.inc"'):
                out.append(os.path.join(d, line.split('"')[1]))
    return out


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


COMMON = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result"]
if os.environ.get("KVEDGE_CHECKS", "0") not in ("", "0"):
    # bounds-check build: launchers verify operand extents against their allocations
    # (a separate object dir so the fast build's objects are not clobbered)
    COMMON.append("-DKVEDGE_CHECKS=1")
    OBJ = os.path.join(ROOT, "build", "obj_checks")
    SO_PATH = os.path.join(PKG, "_C_checks.so")
if os.environ.get("KVEDGE_VARIANT"):
    # A/B variant of the library: extra compile flags (KVEDGE_CFLAGS, e.g. -DKV_GLDS_IL=1),
    # own object dir, linked as kvedge_amd/_C_<variant>.so (load with KVEDGE_LIB=_C_<v>.so)
    _v = os.environ["KVEDGE_VARIANT"]
    COMMON.extend(os.environ.get("KVEDGE_CFLAGS", "").split())
    OBJ = os.path.join(ROOT, "build", "obj_" + _v)
    SO_PATH = os.path.join(PKG, f"_C_{_v}.so")


def build(force: bool = False, jobs: int = 0, verbose: bool = False, asan: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(BIN, exist_ok=True)
    inc, lib, abi = _torch_paths()
    headers = _headers()
    kernel_srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    runtime_srcs = sorted(p for p in glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))
                          if not p.endswith("_main.cpp"))
    bind_srcs = sorted(glob.glob(os.path.join(CSRC, "bindings", "*.cpp")))
    torch_flags = [f"-I{p}" for p in inc] + [
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DUSE_ROCM=1",
        "-D__HIP_PLATFORM_AMD__=1",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
    ]
    py_inc = sysconfig.get_paths()["include"]
    jobs = jobs or min(8, os.cpu_count() or 4)

    tasks = []
    objs = []
    for src in kernel_srcs:
        o = os.path.join(OBJ, os.path.basename(src) + ".o")
        objs.append(o)
        if force or _stale(o, [src] + headers + _incs(src)):
            tasks.append([hipcc(), *COMMON, f"-I{CSRC}/kernels", "-c", src, "-o", o])
    for src in runtime_srcs:
        o = os.path.join(OBJ, os.path.basename(src) + ".o")
        objs.append(o)
        if force or _stale(o, [src] + headers):
            tasks.append([hipcc(), *COMMON, f"-I{CSRC}/runtime", "-c", src, "-o", o])
    for src in bind_srcs:
        o = os.path.join(OBJ, os.path.basename(src) + ".o")
        objs.append(o)
        if force or _stale(o, [src] + headers):
            tasks.append([hipcc(), *COMMON, *torch_flags, f"-I{py_inc}", f"-I{CSRC}/runtime",
                          "-c", src, "-o", o])
    if tasks:
        with cf.ThreadPoolExecutor(jobs) as ex:
            for out in ex.map(_run, tasks):
                if verbose and out.strip():
                    print(out)
    if force or tasks or _stale(SO_PATH, objs):
        _run([hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", SO_PATH,
              f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
              f"-Wl,-rpath,{lib}"])

    # native tools (separate processes; link the system ROCm libs)
    tools = {
        "kv_rccl_bench": (os.path.join(CSRC, "comm", "rccl_bench.cpp"),
                          ["-lrccl"]),
        "kv_runtime_selftest": (os.path.join(CSRC, "runtime", "selftest_main.cpp"), []),
    }
    for name, (src, libs) in tools.items():
        if not os.path.exists(src):
            continue
        out = os.path.join(BIN, name)
        extra_src = runtime_srcs if name == "kv_runtime_selftest" else []
        if force or _stale(out, [src] + extra_src + headers):
            _run([hipcc(), *COMMON, f"-I{CSRC}/runtime", f"-I{CSRC}/kernels", src, *extra_src,
                  "-o", out, f"-L{ROCM}/lib", *libs, f"-Wl,-rpath,{ROCM}/lib"])
    if asan:
        build_asan()
    return SO_PATH


def build_asan() -> str:
    """Host-AddressSanitizer + UBSan build of the native runtime self-test.
    GPU ASan / xnack+ code objects are not available on the MI355X pool, so the
    sanitizers are applied to host code only (`-Xarch_host -fsanitize=...`)."""
    os.makedirs(BIN, exist_ok=True)
    srcs = [os.path.join(CSRC, "runtime", "selftest_main.cpp")] + sorted(
        p for p in glob.glob(os.path.join(CSRC, "runtime", "*.cpp")) if not p.endswith("_main.cpp"))
    out = os.path.join(BIN, "kv_runtime_selftest_asan")
    _run([hipcc(), "-O1", "-g", "-std=c++17", f"--offload-arch={ARCH}",
          "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
          "-Xarch_host", "-fno-omit-frame-pointer", f"-I{CSRC}/runtime", *srcs, "-o", out,
          f"-L{ROCM}/lib", f"-Wl,-rpath,{ROCM}/lib"])
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--checks", action="store_true",
                    help="bounds-check build (-DKVEDGE_CHECKS): set KVEDGE_CHECKS=1 instead "
                         "(must be set before import); this flag only reports it")
    ap.add_argument("--asan", action="store_true",
                    help="also build the host-ASan/UBSan runtime self-test")
    a = ap.parse_args(argv)
    path = build(force=a.force, jobs=a.jobs, verbose=a.verbose, asan=a.asan)
    print(path)


if __name__ == "__main__":
    sys.exit(main())
