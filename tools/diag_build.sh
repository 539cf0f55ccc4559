#!/bin/bash
# Timing-attribution build of the step kernel (-DG2048_DIAG=1: G2048_DIAG_FLAGS removes pieces of the kernel,
# see csrc/g2048.hip).  Loaded instead of the shipped library only through _lib.use_library_for_tools (tools, bench.py --lib).  Never shipped.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG="$ROOT/rl-2048-with-reinforce-and-actor-critic_amd"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DG2048_DIAG=1 -shared -fPIC -I"$ROOT/include" \
  -I"$PKG/csrc" -o "$ROOT/tools/libg2048_diag.so" "$PKG/csrc/g2048.hip" "$PKG/csrc/g2048_policy.hip"
