#!/usr/bin/env bash
# CPU suite under AddressSanitizer + UBSan.  Builds the host-only C++ of the package
# (OBJ import, BVH builders, scene validation / packing: _native.HOST_ONLY) and the CPU oracle with
# -fsanitize=address,undefined,float-cast-overflow (oracle/Makefile asan), preloads gcc's ASan and UBSan
# runtimes into python, points the loaders at the sanitized libraries and runs the "not gpu" tests.
# Any report aborts the run (halt_on_error / -fno-sanitize-recover).  Host-only: no GPU code is
# sanitized (GPU ASan is not available on this pool).
#   tools/sanitize.sh [pytest args...]      default: tests -m "not gpu" -x -q
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
make -s -C "$ROOT/oracle" asan
ASAN_RT="$(gcc -print-file-name=libasan.so)"
UBSAN_RT="$(gcc -print-file-name=libubsan.so)"
export ENSEM3A_HOST_LIB="$ROOT/build/asan/libensem3a_host_asan.so"
export ENSEM3A_ORACLE_LIB="$ROOT/build/asan/liboracle_asan.so"
# leaks: python's own allocations are not ours to report; new/delete and malloc/free mismatches are
export ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1:detect_odr_violation=0:alloc_dealloc_mismatch=1"
export UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1"
# --capture=sys: pytest captures python-level output only, so a sanitizer report (written to fd 2 by the
# native runtime just before it aborts the process) reaches the terminal instead of a discarded capture file
if [ "$#" -eq 0 ]; then set -- tests -m "not gpu" -x -q -p no:cacheprovider; fi
set -- --capture=sys "$@"
cd "$ROOT"
LD_PRELOAD="$ASAN_RT $UBSAN_RT" python -m pytest "$@"
