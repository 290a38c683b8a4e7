"""Builds libgdsm.so (gfx950) in-tree with hipcc, and the test oracle with make.

The shared library lands in gallocy_amd/lib/ so it travels with the repository snapshot to the
GPU box (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIBDIR = PKG / "lib"
LIB = LIBDIR / "libgdsm.so"
SOURCES = ["gdsm_pages.hip", "gdsm_coherence.hip", "gdsm_capi.cpp", "legacy_diff.cpp",
           "gdsm_track.cpp", "gdsm_nw.hip", "gdsm_wire.hip"]
HEADERS = ["gdsm_common.h", "gdsm_launch.h", "gdsm_prof.h", "gdsm_track.h"]
ARCH = os.environ.get("GDSM_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found")


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build_lib(force: bool = False, verbose: bool = False) -> Path:
    deps = [CSRC / s for s in SOURCES] + [CSRC / h for h in HEADERS] + [ROOT / "include" / "gdsm.h"]
    if not force and not _stale(LIB, deps):
        return LIB
    LIBDIR.mkdir(exist_ok=True)
    objs = []
    for s in SOURCES:
        obj = LIBDIR / (Path(s).stem + ".o")
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wall",
               "-I", str(ROOT / "include"), "-I", str(CSRC), "-c", str(CSRC / s), "-o", str(obj)]
        if s.endswith(".cpp"):
            cmd[1:1] = ["-x", "hip"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        objs.append(str(obj))
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *objs,
           "-Wl,--no-undefined"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


def build_oracle(verbose: bool = False) -> None:
    """Test oracle (oracle/liboracle.so) and, when the reference tree exists, oracle/_ref."""
    targets = ["oracle"]
    if Path("/root/reference/gallocy/utils/diff.cpp").exists():
        targets.append("ref")
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), *targets], check=True,
                   stdout=None if verbose else subprocess.DEVNULL)


if __name__ == "__main__":
    build_lib(force="--force" in sys.argv, verbose=True)
    build_oracle(verbose=True)
    print(LIB)
