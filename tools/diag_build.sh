#!/bin/bash
# Timing-attribution build of the step kernel (-DG2048_DIAG=1 on g2048.hip: G2048_DIAG_FLAGS removes pieces of the
# kernel, see csrc/g2048.hip) -> tools/libg2048_dg.so.  Loaded instead of the shipped library only through
# _lib.use_library_for_tools (tools, bench.py --lib).  Never shipped.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT" && python tools/build_variants.py dg=G2048_DIAG=1
