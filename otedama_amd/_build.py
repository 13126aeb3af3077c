"""In-tree build of the native extension ``otedama_amd._native``.

HIP sources (gfx950 kernels + the GPU runtime) are compiled with ``hipcc
--offload-arch=gfx950``; host C++ (SHA-NI SHA-256, scrypt reference, CPU miner,
pybind11 bindings) with ``g++``; everything links into one shared object next
to this file, so it travels with the repo snapshot to the GPU box.

Usage: ``python -m otedama_amd._build [-v] [-j N] [--force]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "native"
ARCH = "gfx950"  # MI355X (CDNA4) only: the kernels use gfx950 instructions (v_bitop3, buffer-load-to-LDS)

HIP_SOURCES = [
    "kernels/sha256d_search.hip",
    "kernels/sha256d_search_v.hip",
    "kernels/scrypt_search.hip",
    "kernels/x11_stages_a.hip",
    "kernels/x11_stages_b.hip",
    "runtime/gpu_miner.hip",
]
CXX_SOURCES = [
    "cpu/sha256_cpu.cpp",
    "cpu/job_prepare.cpp",
    "cpu/aead.cpp",
    "cpu/x11_cpu.cpp",
    "cpu/sv2_frame.cpp",
    "runtime/miner_common.cpp",
    "bindings.cpp",
]


# The node's native RCCL data plane is a module of its own (``otedama_amd._rccl``): only a node rank loads it, so
# librccl is never mapped into the engine, the device processes or the pool.
RCCL_SOURCES = ["runtime/rccl_comm.cpp"]


def ext_path(name: str = "_native") -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return ROOT / "otedama_amd" / f"{name}{suffix}"


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm required to build the gfx950 kernels)")


def _headers() -> list[Path]:
    return sorted(p for p in CSRC.rglob("*.h"))


def _stale(obj: Path, src: Path, deps: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return src.stat().st_mtime > t or any(d.stat().st_mtime > t for d in deps)


def _compile(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")


# Per-source extra hipcc flags. sha256d_search.hip: the K-variant kernels (K up to 16) unroll 60 rounds x K
# states; above LLVM's default pragma-unroll budget the round loop stays rolled and the message schedule and
# state arrays go to scratch (see the kernel's header comment).
EXTRA_FLAGS = {"kernels/sha256d_search.hip": ["-mllvm", "-pragma-unroll-threshold=1000000"],
               "kernels/sha256d_search_v.hip": ["-mllvm", "-pragma-unroll-threshold=1000000"]}


def build(verbose: bool = False, jobs: int | None = None, force: bool = False) -> Path:
    import pybind11

    BUILD.mkdir(parents=True, exist_ok=True)
    hipcc = _hipcc()
    deps = _headers()
    py_inc = sysconfig.get_paths()["include"]
    common = ["-O3", "-std=c++17", "-fPIC", f"-I{CSRC / 'include'}", f"-I{CSRC / 'kernels'}"]
    tasks: list[list[str]] = []
    objs: list[Path] = []
    for rel in HIP_SOURCES:
        src = CSRC / rel
        if not src.exists():
            continue
        obj = BUILD / (rel.replace("/", "_") + ".o")
        objs.append(obj)
        if force or _stale(obj, src, deps):
            tasks.append([hipcc, f"--offload-arch={ARCH}", *common, *EXTRA_FLAGS.get(rel, []), "-c", str(src), "-o",
                          str(obj)])
    for rel in CXX_SOURCES:
        src = CSRC / rel
        if not src.exists():
            continue
        obj = BUILD / (rel.replace("/", "_") + ".o")
        objs.append(obj)
        if force or _stale(obj, src, deps):
            tasks.append(["g++", *common, "-march=x86-64-v2", "-I/opt/rocm/include", f"-I{py_inc}", f"-I{pybind11.get_include()}",
                          "-fvisibility=hidden", "-c", str(src), "-o", str(obj)])
    n = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=n) as ex:
        for f in [ex.submit(_compile, t, verbose) for t in tasks]:
            f.result()
    out = ext_path()
    if force or tasks or not out.exists() or any(o.stat().st_mtime > out.stat().st_mtime for o in objs):
        tmp = out.with_suffix(".tmp.so")
        # DT_NEEDED is the sonames libamdhip64.so.7 / libhsa-runtime64.so.1,
        # which torch's bundled runtime also carries: ops.native imports torch
        # first, so the extension binds to the runtime already in the process
        # (two HIP/HSA runtimes in one process fail to enumerate the GPU).
        link = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp), "-lpthread", "-lcrypto",
                "-L/opt/rocm/lib", "-lrocprofiler-sdk-roctx", "-lhsa-runtime64"]
        _compile(link, verbose)
        os.replace(tmp, out)
    build_rccl(verbose, force, hipcc, common, py_inc, pybind11.get_include())
    return out


def build_rccl(verbose: bool, force: bool, hipcc: str, common: list[str], py_inc: str, pyb_inc: str) -> Path:
    """``otedama_amd._rccl``: host code only (RCCL + the HIP runtime API, no kernels), compiled as HIP for gfx950 like
    the miner runtime, linked to librccl."""
    out = ext_path("_rccl")
    objs, tasks = [], []
    deps = _headers()
    for rel in RCCL_SOURCES:
        src = CSRC / rel
        obj = BUILD / (rel.replace("/", "_") + ".o")
        objs.append(obj)
        if force or _stale(obj, src, deps):
            tasks.append([hipcc, f"--offload-arch={ARCH}", *common, "-I/opt/rocm/include", f"-I{py_inc}",
                          f"-I{pyb_inc}", "-fvisibility=hidden", "-x", "hip", "-c", str(src), "-o", str(obj)])
    for t in tasks:
        _compile(t, verbose)
    if force or tasks or not out.exists() or any(o.stat().st_mtime > out.stat().st_mtime for o in objs):
        tmp = out.with_suffix(".tmp.so")
        _compile([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp), "-L/opt/rocm/lib", "-lrccl",
                  "-lamdhip64"], verbose)
        os.replace(tmp, out)
    return out


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args(argv)
    p = build(a.verbose, a.jobs, a.force)
    print(p)
    return 0


if __name__ == "__main__":
    sys.exit(main())
