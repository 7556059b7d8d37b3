#!/bin/bash
# HBM traffic of the skim kernel on config 2 (tools/skim_ab.py): separate
# rocprofv3 --pmc passes for FETCH_SIZE and WRITE_SIZE (kernel trace only).
# Outputs under gpurun_out/skim_pmc/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=$PWD/gpurun_out/skim_pmc; mkdir -p "$OUT"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$OUT/$c" -o run -- python3 "$OLDPWD/tools/skim_ab.py" 2) > "$OUT/$c.log" 2>&1 || { echo "pmc $c failed $?"; tail -5 "$OUT/$c.log"; exit 3; }
done
echo done
