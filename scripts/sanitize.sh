#!/usr/bin/env bash
# Host AddressSanitizer + UBSan run of the CPU tests (the reference has none; its own
# diff() has a 1-byte overflow at diff.cpp:139-140 and reads _matrix[-1] at :146-152).
# Builds gallocy_amd/lib_san/libgdsm.so and oracle/_san/liboracle.so (clang, -fsanitize=
# address,undefined on host code only) and runs tests/test_track.py, test_capi.py and
# test_oracle.py against them. CPU only; never run on the GPU box.
set -euo pipefail
cd "$(dirname "$0")/.."
python gallocy_amd/build.py --sanitize > /dev/null 2>&1 || { echo "sanitizer build failed" >&2; exit 1; }
ASAN_RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
# handle_segv=0: the write-fault tracker owns SIGSEGV (and chains unrelated faults to the
# default action, which tests/test_track.py checks); leaks of the Python interpreter are not ours.
export ASAN_OPTIONS=detect_leaks=0:handle_segv=0:halt_on_error=1:abort_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
export GDSM_LIB=gallocy_amd/lib_san/libgdsm.so GDSM_ORACLE_LIB=oracle/_san/liboracle.so
export GDSM_NO_TORCH=1
# the runtime is live and the instrumented builds are the ones loaded
LD_PRELOAD="$ASAN_RT" python -c "
import ctypes
from gallocy_amd import _lib
from oracle import oracle
ctypes.CDLL(None).__asan_report_load1
assert str(_lib.LIB_PATH).endswith('lib_san/libgdsm.so') and '_san' in str(oracle.LIB)
print('asan+ubsan:', _lib.LIB_PATH, oracle.LIB)"
LD_PRELOAD="$ASAN_RT" python -m pytest -q -p no:cacheprovider tests/test_track.py tests/test_capi.py \
  tests/test_oracle.py "$@"
