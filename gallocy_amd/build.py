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
           "gdsm_track.cpp", "gdsm_nw.hip", "gdsm_wire.hip", "gdsm_exchange.cpp", "gdsm_route.hip", "gdsm_probe.hip"]
HEADERS = ["gdsm_common.h", "gdsm_launch.h", "gdsm_prof.h", "gdsm_track.h", "gdsm_ctx.h"]
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
               "-Werror=inline-asm", "-I", str(ROOT / "include"), "-I", str(CSRC), "-c", str(CSRC / s), "-o", str(obj)]
        if s.endswith(".cpp"):
            cmd[1:1] = ["-x", "hip"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        objs.append(str(obj))
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *objs,
           "-ldl", "-Wl,--no-undefined"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


SAN_DIR = PKG / "lib_san"
SAN_FLAGS = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
             "-Xarch_host", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-g"]


def build_sanitized(verbose: bool = False) -> Path:
    """Host AddressSanitizer + UBSan build of libgdsm.so (gallocy_amd/lib_san/) and of the C
    oracle (oracle/_san/liboracle.so), both with the clang that hipcc drives, so one runtime
    (libclang_rt.asan) serves the process. The device code is compiled as usual (GPU sanitizers
    are not used). Run the CPU tests against it with scripts/sanitize.sh."""
    SAN_DIR.mkdir(exist_ok=True)
    objs = []
    for s in SOURCES:
        obj = SAN_DIR / (Path(s).stem + ".o")
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O1", "-fPIC", "-std=c++17", *SAN_FLAGS,
               "-I", str(ROOT / "include"), "-I", str(CSRC), "-c", str(CSRC / s), "-o", str(obj)]
        if s.endswith(".cpp"):
            cmd[1:1] = ["-x", "hip"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        objs.append(str(obj))
    lib = SAN_DIR / "libgdsm.so"
    subprocess.run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC",
                    "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
                    "-shared-libsan", "-o", str(lib), *objs, "-ldl"], check=True)
    clang = Path(_hipcc()).resolve().parent.parent / "lib" / "llvm" / "bin" / "clang"
    if not clang.exists():
        clang = Path("/opt/rocm/lib/llvm/bin/clang")
    (ROOT / "oracle" / "_san").mkdir(exist_ok=True)
    subprocess.run([str(clang), "-std=c99", "-O1", "-g", "-fPIC", "-shared", "-Wall",
                    "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                    "-shared-libsan", "-fno-omit-frame-pointer",
                    "-fopenmp", "-o", str(ROOT / "oracle" / "_san" / "liboracle.so"),
                    str(ROOT / "oracle" / "gdsm_oracle.c"),
                    str(ROOT / "oracle" / "gdsm_oracle_bench.c")], check=True)
    return lib


REPLAY = LIBDIR / "libgdsm_replay.so"


def build_replay(verbose: bool = False) -> Path:
    """The C++ round loop of config 5's replay (gallocy_amd/native/replay.cpp) over libgdsm.so's
    C ABI, for bench.py / replay.py (a bench driver, not part of libgdsm)."""
    src = PKG / "native" / "replay.cpp"
    if not _stale(REPLAY, [src, ROOT / "include" / "gdsm.h", LIB]):
        return REPLAY
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-fPIC", "-shared",
           "-I", str(ROOT / "include"), str(src), "-L", str(LIBDIR), "-lgdsm",
           "-Wl,-rpath,$ORIGIN", "-Wl,--no-undefined", "-pthread", "-o", str(REPLAY)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return REPLAY


def build_test_drivers(verbose: bool = False) -> None:
    """Compiled C++ callers of libgdsm.so used by the tests (tests/cpp/, output in _build/)."""
    subprocess.run(["make", "-s", "-C", str(ROOT / "tests" / "cpp")], check=True,
                   stdout=None if verbose else subprocess.DEVNULL)


def build_oracle(verbose: bool = False) -> None:
    """Test oracle (oracle/liboracle.so) and, when the reference tree exists, oracle/_ref."""
    targets = ["oracle"]
    if Path("/root/reference/gallocy/utils/diff.cpp").exists():
        targets += ["ref", "caller", "layout"]
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), *targets], check=True,
                   stdout=None if verbose else subprocess.DEVNULL)


if __name__ == "__main__":
    if "--sanitize" in sys.argv:
        print(build_sanitized(verbose=True))
        sys.exit(0)
    build_lib(force="--force" in sys.argv, verbose=True)
    build_replay(verbose=True)
    build_test_drivers(verbose=True)
    build_oracle(verbose=True)
    print(LIB)
