"""Build the in-tree HIP kernel library for gfx950 (MI355X).

Every ``csrc/*.hip`` file is compiled with ``hipcc --offload-arch=gfx950`` into an object and
linked into ``_lib/libmfa_hip.so``.  The library exposes a plain C ABI (raw device pointers +
``hipStream_t``) consumed through :mod:`ctypes` by :mod:`._native`, so the build needs neither
torch headers nor a JIT cache: the ``.so`` lives in-tree and travels with the repository
snapshot to the GPU box.

Usage::

    python -m llm_driven_multi_factor_model_amd._build [--force] [-j 8] [--ab]

``--ab`` builds the A/B library ``_lib/ab/libmfa_hip.so`` with ``-DMFA_AB=1``: the kernel
variants that lost their measured A/B comparisons and the timing-only ablations, which the
default (production) library does not contain.  The ``tools/`` A/B scripts load it through
``MFA_HIP_LIB=.../_lib/ab/libmfa_hip.so``; tests of those variants skip on the production build.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import re
import shutil
import subprocess
import sys
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR / "csrc"
OBJ_DIR = PKG_DIR / "_lib" / "obj"
LIB_PATH = PKG_DIR / "_lib" / "libmfa_hip.so"
AB_OBJ_DIR = PKG_DIR / "_lib" / "ab" / "obj"
AB_LIB_PATH = PKG_DIR / "_lib" / "ab" / "libmfa_hip.so"
HOST_SRC = PKG_DIR / "csrc_host"
HOST_LIB_PATH = PKG_DIR / "_lib" / "libmfa_host.so"
ARCH = os.environ.get("MFA_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (set HIPCC or install ROCm at /opt/rocm)")


def _flags(ab: bool = False) -> list[str]:
    return [
        *(["-DMFA_AB=1"] if ab else []),
        f"--offload-arch={ARCH}",
        "-O3",
        "-std=c++20",
        "-fPIC",
        "-ffp-contract=fast",
        "-munsafe-fp-atomics",
        f"-I{CSRC}",
    ]


def sources() -> list[Path]:
    return sorted(CSRC.glob("*.hip"))


def _local_includes(src: Path, seen: set[Path] | None = None) -> set[Path]:
    """Headers of csrc/ that `src` includes, transitively (#include "x.h")."""
    seen = set() if seen is None else seen
    for m in re.finditer(r'^\s*#\s*include\s+"([^"]+)"', src.read_text(), re.M):
        h = CSRC / m.group(1)
        if h.exists() and h not in seen:
            seen.add(h)
            _local_includes(h, seen)
    return seen


def _stale(src: Path, obj: Path, headers: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    deps = _local_includes(src) & set(headers)
    return src.stat().st_mtime > t or any(h.stat().st_mtime > t for h in deps)


def _compile(src: Path, obj: Path, ab: bool = False) -> tuple[Path, str]:
    cmd = [_hipcc(), *_flags(ab), "-c", str(src), "-o", str(obj)]
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{p.stderr}")
    return obj, p.stderr


def build_host(force: bool = False, verbose: bool = False) -> Path:
    """Native host runtime (CSV/panel IO, as-of joins): plain C++17 + pthreads, C ABI."""
    srcs = sorted(HOST_SRC.glob("*.cpp"))
    if not srcs:
        return HOST_LIB_PATH
    if not force and HOST_LIB_PATH.exists() and all(
            s.stat().st_mtime <= HOST_LIB_PATH.stat().st_mtime for s in srcs):
        return HOST_LIB_PATH
    HOST_LIB_PATH.parent.mkdir(parents=True, exist_ok=True)
    cxx = os.environ.get("CXX", shutil.which("g++") or "c++")
    tmp = HOST_LIB_PATH.with_suffix(".so.tmp")
    cmd = [cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", *map(str, srcs), "-o", str(tmp)]
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0:
        raise RuntimeError(f"host build failed:\n{p.stderr}")
    os.replace(tmp, HOST_LIB_PATH)
    if verbose:
        print(f"[mfa-build] linked {HOST_LIB_PATH}", file=sys.stderr)
    return HOST_LIB_PATH


def build(force: bool = False, jobs: int | None = None, verbose: bool = False,
          ab: bool = False) -> Path:
    """Compile all kernels (incrementally) and link the shared library; returns its path.
    ``ab``: the A/B library (MFA_AB=1) in ``_lib/ab/`` instead of the production one."""
    build_host(force=force, verbose=verbose)
    obj_dir, lib_path = (AB_OBJ_DIR, AB_LIB_PATH) if ab else (OBJ_DIR, LIB_PATH)
    obj_dir.mkdir(parents=True, exist_ok=True)
    headers = sorted(CSRC.rglob("*.h"))   # csrc/ab/*.h: the A/B-only kernels (MFA_AB builds)
    srcs = sources()
    objs = [obj_dir / (s.stem + ".o") for s in srcs]
    todo = [(s, o) for s, o in zip(srcs, objs) if force or _stale(s, o, headers)]
    jobs = jobs or min(8, max(1, (os.cpu_count() or 2)))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=min(jobs, len(todo))) as ex:
            for obj, err in ex.map(lambda so: _compile(*so, ab=ab), todo):
                if verbose:
                    print(f"[mfa-build] compiled {obj.name}", file=sys.stderr)
    relink = force or bool(todo) or not lib_path.exists() or any(
        o.stat().st_mtime > lib_path.stat().st_mtime for o in objs)
    if relink:
        tmp = lib_path.with_suffix(".so.tmp")
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp)]
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"link failed:\n{p.stderr}")
        os.replace(tmp, lib_path)
        if verbose:
            print(f"[mfa-build] linked {lib_path}", file=sys.stderr)
    return lib_path


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--ab", action="store_true", help="A/B library with the losing variants")
    a = ap.parse_args(argv)
    print(build(force=a.force, jobs=a.jobs, verbose=True, ab=a.ab))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
