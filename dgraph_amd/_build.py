"""In-tree build of the native library ``dgraph_amd/_C.so`` for gfx950.

Replaces the reference's scikit-build/CMake CUDA build (CMakeLists.txt:1-192,
pyproject.toml:1-66). Every ``csrc/**/*.hip`` translation unit is compiled by
``hipcc --offload-arch=gfx950`` (device + host), every ``csrc/**/*.cpp`` unit as host
C++ against the PyTorch-ROCm headers, and the objects are linked into one shared
library registered with the dispatcher (``TORCH_LIBRARY(dgraph_amd, ...)``).

The library links against the HIP runtime and RCCL that ship inside the torch wheel
(same SONAMEs as /opt/rocm), so exactly one HIP runtime lives in the process.

Usage: ``python -m dgraph_amd._build`` (incremental; ``--force`` rebuilds all).
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

REPO = Path(__file__).resolve().parent.parent
CSRC = REPO / "csrc"
OBJ_DIR = REPO / "build" / "obj"
TARGET = Path(__file__).resolve().parent / "_C.so"
ARCH = os.environ.get("DGRAPH_OFFLOAD_ARCH", "gfx950")
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))


def _torch_dirs():
    import torch  # noqa: F401  (deferred: build() must not need a GPU)

    root = Path(torch.__file__).resolve().parent
    inc = [root / "include", root / "include" / "torch" / "csrc" / "api" / "include"]
    return inc, root / "lib"


def _hipcc() -> str:
    for cand in (ROCM / "bin" / "hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return str(cand)
    raise RuntimeError("hipcc not found (set ROCM_PATH)")


def _common_flags():
    import torch

    inc, _ = _torch_dirs()
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    flags = [
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-Wno-unused-result",
        "-Wno-deprecated-declarations",
        f"-I{CSRC}",
        f"-I{ROCM / 'include'}",
    ]
    flags += [f"-isystem{p}" for p in inc]
    return flags


def _sources():
    srcs = sorted(CSRC.rglob("*.hip")) + sorted(CSRC.rglob("*.cpp"))
    srcs = [s for s in srcs if not s.name.startswith("test_")]  # host test drivers (main())
    headers = sorted(CSRC.rglob("*.h")) + sorted(CSRC.rglob("*.hpp"))
    return srcs, headers


def _obj_for(src: Path) -> Path:
    rel = src.relative_to(CSRC).with_suffix(".o")
    return OBJ_DIR / str(rel).replace(os.sep, "__")


def _compile(src: Path, force: bool, newest_header: float) -> Path:
    obj = _obj_for(src)
    if (
        not force
        and obj.exists()
        and obj.stat().st_mtime >= max(src.stat().st_mtime, newest_header)
    ):
        return obj
    obj.parent.mkdir(parents=True, exist_ok=True)
    cmd = [_hipcc()] + _common_flags()
    if src.suffix == ".hip":
        cmd += [f"--offload-arch={ARCH}", "-x", "hip", "-c", str(src), "-o", str(obj)]
    else:
        cmd += ["-x", "c++", "-c", str(src), "-o", str(obj)]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    return obj


def build(force: bool = False, jobs: int | None = None, verbose: bool = True) -> Path:
    srcs, headers = _sources()
    newest_header = max((h.stat().st_mtime for h in headers), default=0.0)
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, newest_header), srcs))
    newest_obj = max(o.stat().st_mtime for o in objs)
    if not force and TARGET.exists() and TARGET.stat().st_mtime >= newest_obj:
        if verbose:
            print(f"[dgraph_amd._build] up to date: {TARGET}")
        return TARGET
    _, torch_lib = _torch_dirs()
    cmd = (
        [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}"]
        + [str(o) for o in objs]
        + [
            f"-L{torch_lib}",
            "-lc10",
            "-lc10_hip",
            "-ltorch",
            "-ltorch_cpu",
            "-ltorch_hip",
            "-lamdhip64",
            "-lrccl",
            f"-Wl,-rpath,{torch_lib}",
            "-o",
            str(TARGET),
        ]
    )
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    if verbose:
        print(f"[dgraph_amd._build] built {TARGET} from {len(objs)} objects")
    return TARGET


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.jobs)


if __name__ == "__main__":
    main()
