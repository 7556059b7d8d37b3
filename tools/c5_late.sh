#!/bin/bash
# Does the LDS-staged tile change after the staging barrier? (TGPU_SPEC_LATE)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for v in "#define TGPU_SPEC_LATE 1
#define TGPU_SPEC_CHECK 1" "#define TGPU_SPEC_LATE 1
#define TGPU_SPEC_CHECK 1
#define TGPU_SPEC_REGSTAGE 1"; do
  TGPU_INDEX_TIMING=2 TGPU_JIT_DEFINES="$v" timeout -k 10 200 python tools/c5_time.py --variants 1 --reps 12 --stats > gpurun_out/c5late.log 2>&1 || exit 1
  echo "[$v]" | tr '\n' ' '; echo
  grep "spec check" gpurun_out/c5late.log | sort | uniq -c | sort -rn | head -8
done
