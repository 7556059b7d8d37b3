#!/bin/bash
# Config-5 decode call under schema-compiler defines (VARIANTS, one per line;
# the empty line is the default build), each in its own process.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
while IFS= read -r v; do
  TGPU_JIT_DEFINES="$v" timeout -k 10 200 python tools/c5_time.py --sync-before --variants 1 --reps 6 > gpurun_out/c5v.log 2>&1 || { echo "failed $?"; tail -5 gpurun_out/c5v.log; exit 2; }
  echo "[$v] $(tail -1 gpurun_out/c5v.log)"
done <<< "${VARIANTS:-}"
