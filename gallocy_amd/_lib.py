"""Loads libgdsm.so and declares its C-ABI (include/gdsm.h) for ctypes.

There is no fallback: if the library is missing the import fails loudly. torch, when installed,
is imported first so that libgdsm binds to the same HIP runtime instance torch uses (both ship a
`libamdhip64.so.7`; loading ours first would put two HIP runtimes in one process).
"""
from __future__ import annotations

import ctypes as C
import errno
import os
from pathlib import Path

if os.environ.get("GDSM_NO_TORCH") != "1":  # share torch's HIP runtime when torch is present
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is optional for the C-ABI itself
        torch = None

# GDSM_LIB: another build of the same library, e.g. the host-sanitizer build
# (gallocy_amd/lib_san/libgdsm.so, scripts/sanitize.sh).
LIB_PATH = Path(os.environ.get("GDSM_LIB") or
                Path(__file__).resolve().parent / "lib" / "libgdsm.so").resolve()

u8p = C.POINTER(C.c_uint8)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)
vp = C.c_void_p


class GdsmRuns(C.Structure):
    _fields_ = [("n", C.c_uint64), ("rec_off", vp), ("data", vp), ("cap", C.c_uint64),
                ("n_cap", C.c_uint64), ("owned", C.c_uint32), ("_pad", C.c_uint32)]


# name -> (restype, argtypes)
SIGNATURES = {
    "gdsm_version": (C.c_char_p, []),
    "gdsm_tune": (C.c_int, [C.c_char_p, C.c_int64]),
    "gdsm_debug_fail_alloc": (C.c_int, [vp, C.c_int]),
    "gdsm_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "gdsm_init": (C.c_int, [C.POINTER(vp), C.c_int, C.c_uint64, C.c_uint32]),
    "gdsm_fini": (C.c_int, [vp]),
    "gdsm_arena": (C.c_int, [vp, C.c_int, C.POINTER(vp)]),
    "gdsm_n_pages": (C.c_uint64, [vp]),
    "gdsm_stream": (vp, [vp]),
    "gdsm_sync": (C.c_int, [vp]),
    "gdsm_upload": (C.c_int, [vp, C.c_int, C.c_uint64, C.c_uint64, vp]),
    "gdsm_download": (C.c_int, [vp, C.c_int, C.c_uint64, C.c_uint64, vp]),
    "gdsm_reserve": (C.c_int, [vp, C.c_uint64, C.c_uint64]),
    "gdsm_dev_alloc": (C.c_int, [vp, C.c_uint64, C.POINTER(vp)]),
    "gdsm_dev_free": (C.c_int, [vp, vp]),
    "gdsm_memcpy_h2d": (C.c_int, [vp, vp, vp, C.c_uint64]),
    "gdsm_memcpy_d2h": (C.c_int, [vp, vp, vp, C.c_uint64]),
    "gdsm_memcpy_d2d": (C.c_int, [vp, vp, vp, C.c_uint64]),
    "gdsm_memcpy_batch": (C.c_int, [vp, vp, C.c_uint64]),
    "gdsm_capture_begin": (C.c_int, [vp]),
    "gdsm_capture_join": (C.c_int, [vp, vp]),
    "gdsm_capture_end": (C.c_int, [vp, C.POINTER(vp)]),
    "gdsm_graph_launch": (C.c_int, [vp, vp]),
    "gdsm_graph_destroy": (C.c_int, [vp]),
    "gdsm_prof_enable": (C.c_int, [vp, C.c_int]),
    "gdsm_prof_read": (C.c_int, [vp, C.POINTER(C.c_double), u64p]),
    "gdsm_rounds": (C.c_int, [vp, vp, C.c_uint32, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "gdsm_rounds": (C.c_int, [vp, vp, C.c_uint32, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "gdsm_probe_ceiling": (C.c_int, [vp, C.c_int, vp, vp, vp, C.c_uint64, C.c_int,
                                     C.POINTER(C.c_float), C.POINTER(C.c_float)]),
    "gdsm_gen_pages": (C.c_int, [vp, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int,
                                 C.c_uint32]),
    "gdsm_gen_pages_raw": (C.c_int, [vp, vp, vp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                     C.c_int, C.c_uint32, vp]),
    "gdsm_twin": (C.c_int, [vp, vp, C.c_uint64]),
    "gdsm_runs_alloc": (C.c_int, [vp, C.c_uint64, C.c_uint64, C.POINTER(GdsmRuns)]),
    "gdsm_runs_free": (C.c_int, [vp, C.POINTER(GdsmRuns)]),
    "gdsm_diff": (C.c_int, [vp, vp, C.c_uint64, C.POINTER(GdsmRuns)]),
    "gdsm_diff_apply": (C.c_int, [vp, vp, C.c_uint64, C.POINTER(GdsmRuns), C.c_int]),
    "gdsm_diff_apply_ids": (C.c_int, [vp, vp, C.c_uint64, C.POINTER(GdsmRuns), C.c_int, vp]),
    "gdsm_release": (C.c_int, [vp, vp, C.c_uint64, C.POINTER(GdsmRuns), C.c_int, vp, C.c_uint32]),
    "gdsm_diff_split": (C.c_int, [vp, vp, C.c_uint32, C.POINTER(GdsmRuns)]),
    "gdsm_runs_total": (C.c_int, [vp, C.POINTER(GdsmRuns), C.POINTER(C.c_uint64)]),
    "gdsm_apply": (C.c_int, [vp, C.c_int, vp, C.POINTER(GdsmRuns)]),
    "gdsm_apply_async": (C.c_int, [vp, C.c_int, vp, C.POINTER(GdsmRuns)]),
    "gdsm_diff_workspace_bytes": (C.c_uint64, [C.c_uint64]),
    "gdsm_diff_raw": (C.c_int, [vp, vp, vp, C.c_uint64, vp, vp, C.c_uint64, vp, C.c_uint64, vp]),
    "gdsm_diff_apply_raw": (C.c_int, [vp, vp, vp, vp, C.c_uint64, vp, vp, C.c_uint64, vp,
                                      C.c_uint64, vp]),
    "gdsm_apply_raw": (C.c_int, [vp, vp, C.c_uint64, vp, vp, vp, vp]),
    "gdsm_twin_raw": (C.c_int, [vp, vp, vp, C.c_uint64, vp]),
    "gdsm_coh_init": (C.c_int, [vp, C.c_uint32]),
    "gdsm_coherence_batch": (C.c_int, [vp, vp, C.c_uint64, u64p]),
    "gdsm_coherence_batch_async": (C.c_int, [vp, vp, C.c_uint64, vp]),
    "gdsm_coh_download": (C.c_int, [vp, vp, vp]),
    "gdsm_coh_upload": (C.c_int, [vp, vp, vp]),
    "gdsm_gen_events": (C.c_int, [vp, vp, vp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32,
                                  C.c_uint32]),
    "gdsm_nw_diff": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(C.c_void_p), C.c_char_p,
                               C.c_size_t, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
    "gdsm_set_allocator": (C.c_int, [vp, vp]),
    "gdsm_nw_diff_batch": (C.c_int, [vp, vp, vp, vp, vp, C.c_uint64, C.c_uint32, vp, vp, vp]),
    "gdsm_set_diff_device": (C.c_int, [vp, C.c_uint64]),
    "gdsm_wire_size": (C.c_uint64, [C.c_uint64, C.c_uint64]),
    "gdsm_wire_encode": (C.c_int, [vp, vp, C.POINTER(GdsmRuns), vp, C.c_uint64, u64p]),
    "gdsm_wire_decode": (C.c_int, [vp, C.c_char_p, C.c_uint64, vp, C.POINTER(GdsmRuns), u64p]),
    "gdsm_wire_apply": (C.c_int, [vp, C.c_int, C.c_char_p, C.c_uint64, u64p]),
    "gdsm_track_begin": (C.c_int, [C.POINTER(vp), vp, C.c_uint64]),
    "gdsm_track_dirty": (C.c_int, [vp, vp, C.c_uint64, u64p]),
    "gdsm_track_twin": (C.c_int, [vp, C.POINTER(vp)]),
    "gdsm_track_faults": (C.c_int, [vp, u64p]),
    "gdsm_track_rearm": (C.c_int, [vp]),
    "gdsm_track_end": (C.c_int, [vp]),
    "gdsm_track_diff": (C.c_int, [vp, vp, C.POINTER(GdsmRuns), vp, u64p]),
    "gdsm_comm_unique_id": (C.c_int, [vp]),
    "gdsm_comm_init": (C.c_int, [C.POINTER(vp), vp, C.c_int, C.c_int, vp]),
    "gdsm_comm_fini": (C.c_int, [vp]),
    "gdsm_comm_size": (C.c_int, [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "gdsm_comm_init_loopback": (C.c_int, [C.POINTER(vp), C.POINTER(vp), C.c_int]),
    "gdsm_comm_agree": (C.c_int, [vp, vp, u64p]),
    "gdsm_route_events": (C.c_int, [vp, vp, vp, C.c_uint64, C.c_uint64, vp, C.c_uint64, u64p]),
    "gdsm_coherence_notify": (C.c_int, [vp, vp, vp, C.c_uint64, C.c_uint64, vp, vp, C.c_uint64,
                                        u64p]),
    "gdsm_exchange": (C.c_int, [vp, vp, C.POINTER(GdsmRuns), C.POINTER(vp), C.POINTER(GdsmRuns),
                                C.POINTER(vp), C.c_int, C.c_uint32]),
}
# The legacy C++ symbol (gallocy/include/gallocy/utils/diff.h:9-11), exported unmangled-equal.
LEGACY_DIFF_SYMBOL = "_Z4diffPKcmRPcS0_mS2_"

_lib = None


class GdsmError(OSError):
    pass


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ImportError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; "
                          f"g.build()'` (hipcc, gfx950) first")
    lib = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str = "") -> int:
    if rc < 0:
        code = -rc
        raise GdsmError(code, f"{what}: {os.strerror(code)} ({errno.errorcode.get(code, code)})")
    return rc
