#!/bin/bash
# Spec kernel time per JIT variant (rocprofv3 --stats over tools/c5_time.py),
# and each variant's late-write / stuck-tile diagnostics.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  (cd /tmp && TGPU_JIT_DEFINES="$v" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/gpurun_out/vp$i" -o run -- python3 "$OLDPWD/tools/c5_time.py" --variants 1 --reps 6) > gpurun_out/vp$i.log 2>&1 || { tail -5 gpurun_out/vp$i.log; exit 1; }
  f=$(find gpurun_out/vp$i -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$v" <<'PY'
import csv, sys
rows = {r["Name"]: r for r in csv.DictReader(open(sys.argv[1]))}
def ms(k):
    for n, r in rows.items():
        if n.startswith(k): return float(r["AverageNs"]) / 1e6
    return float("nan")
print("[%s] spec %.3f ms, cont %.3f, copy %.3f, decode %.3f" % (sys.argv[2].replace("\n", " "), ms("tgpu_jit_index_spec"), ms("void tgpu::(anonymous namespace)::index_cont"), ms("tgpu::(anonymous namespace)::index_starts_copy"), ms("tgpu_jit_decode")))
PY
  TGPU_INDEX_TIMING=2 TGPU_JIT_DEFINES="$v
#define TGPU_SPEC_LATE 1" timeout -k 10 200 python tools/c5_time.py --variants 1 --reps 8 --stats > gpurun_out/vpl$i.log 2>&1 || exit 1
  echo "   late-write tiles/threads per call: $(grep -o 'barrier [0-9]*' gpurun_out/vpl$i.log | awk '{print $2}' | tr '\n' ' ')  stuck calls: $(grep -c "'partial': [1-9]" gpurun_out/vpl$i.log)"
done
