#!/bin/bash
# Stuck-tile counts of the candidate speculation under JIT variants (A/B).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for v in "$@"; do
  TGPU_JIT_DEFINES="$v" timeout -k 10 200 python tools/c5_time.py --variants 1 --reps 12 --stats > gpurun_out/c5st.log 2>&1 || exit 1
  echo "[$v] $(grep -c "'partial': [1-9]" gpurun_out/c5st.log) calls with stuck tiles of $(grep -c 'rep ' gpurun_out/c5st.log); $(grep 'decode wall' gpurun_out/c5st.log)"
done
