#!/bin/bash
# Nested-container leg under rocprofv3 (kernel stats) and its bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=$PWD/gpurun_out/pn${TAG:+_$TAG}; mkdir -p "$OUT"
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o n -- python3 "$OLDPWD/bench.py" --config 4 --steps 1 --warmup 1 --no-cpu-baseline --no-copy-ceiling --nested) > "$OUT/out.json" 2> "$OUT/err" || { echo "prof failed"; tail -20 "$OUT/err"; exit 2; }
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats.csv"
python3 - "$OUT/kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:10]:
    print("%-60s n=%-4s avg=%.3f ms" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
python3 -c "import json; d=json.loads(open('$OUT/out.json').read().strip().splitlines()[-1]); n=d['nested']; print('nested enc', n['encode_ms'], 'dec', n['decode_ms'])"
