#!/bin/bash
# Late LDS writes (TGPU_SPEC_LATE) of the index speculation per staging variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for v in "$@"; do
  TGPU_INDEX_TIMING=2 TGPU_JIT_DEFINES="$v
#define TGPU_SPEC_LATE 1" timeout -k 10 200 python tools/c5_time.py --variants 1 --reps 8 --stats > gpurun_out/c5la.log 2>&1 || { tail -3 gpurun_out/c5la.log; exit 1; }
  echo "[$v] late: $(grep -o 'barrier [0-9]*' gpurun_out/c5la.log | awk '{print $2}' | tr '\n' ' ') stuck calls: $(grep -c "'partial': [1-9]" gpurun_out/c5la.log)" | tr '\n' ' '; echo
done
