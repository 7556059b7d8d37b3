#!/bin/bash
# Config-5 decode call: candidate-list vs slice speculation (A/B by
# TGPU_JIT_DEFINES), then SQ counters of the default build (NAME=sq_c5).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for v in "" "#define TGPU_SLICE_SPEC 1" "" "#define TGPU_SLICE_SPEC 1"; do
  TGPU_JIT_DEFINES="$v" timeout -k 10 200 python tools/c5_time.py --variants 1 --reps 8 > gpurun_out/c5spec.log 2>&1 || exit 1
  echo "[$v] $(grep 'decode wall' gpurun_out/c5spec.log)"
done
[ -n "$SQ" ] && NAME=sq_c5 PROG="tools/c5_time.py --variants 1 --reps 1" bash tools/pmc_sq.sh | grep -A30 "tgpu_jit_index_spec"
exit 0
