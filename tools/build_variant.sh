#!/bin/bash
# A diagnostics build of libtgpu.so with extra -D flags, out of tree:
#   tools/build_variant.sh scratch/dbg -DTGPU_PLAN_STALE_CHECK
# then TGPU_LIB_PATH=scratch/dbg/libtgpu.so for the run (fbthrift_amd/_lib.py).
cd "$(dirname "$0")/.." || exit 1
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT/obj"
make -s -j8 -C fbthrift_amd/csrc OBJDIR="$OUT/obj" LIB="$OUT/libtgpu.so" \
  FLAGS="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -Wall -Wno-unused-function $*"
