#!/bin/bash
# Stuck tiles of the candidate speculation: default; a host sync between the
# encode and the decode call (--sync-before); kernels serialized by HIP
# (AMD_SERIALIZE_KERNEL=3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
run() {
  timeout -k 10 200 "$@" > gpurun_out/c5ov.log 2>&1 || { tail -5 gpurun_out/c5ov.log; exit 1; }
  echo "$(grep -c "'partial': [1-9]" gpurun_out/c5ov.log) calls with stuck tiles of $(grep -c 'rep ' gpurun_out/c5ov.log); $(grep 'decode wall' gpurun_out/c5ov.log)"
}
echo -n "default: "; run python tools/c5_time.py --variants 1 --reps 12 --stats
echo -n "sync before decode: "; run python tools/c5_time.py --variants 1 --reps 12 --stats --sync-before
echo -n "AMD_SERIALIZE_KERNEL=3: "; AMD_SERIALIZE_KERNEL=3 run python tools/c5_time.py --variants 1 --reps 12 --stats
