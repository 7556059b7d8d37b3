#!/bin/bash
# One GPU call: the selected tests (TESTS), then bench lines for CONFIGS with
# their kernel summaries (rocprofv3 --stats). Outputs under gpurun_out/q_$TAG.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=$PWD/gpurun_out/q${TAG:+_$TAG}; mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TLIMIT:-600} python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 2; }
  tail -2 "$OUT/pytest.log"
fi
for c in ${CONFIGS:-3 5}; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-copy-ceiling $BENCH_ARGS > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err" || { echo "bench c$c failed"; tail -20 "$OUT/bench_c$c.err"; exit 3; }
  python -c "import json; d=json.load(open('$OUT/bench_c$c.json')); r=d['roofline']; print('c$c value', d['value'], 'dec ms', r['avg_launch_ms'], 'frac', r['frac'], 'enc ms', r['encode']['avg_launch_ms'], 'enc frac', r['encode']['frac'])"
  if [ -n "$PROF" ]; then
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c$c" -o run -- python3 "$OLDPWD/bench.py" --config $c --steps 5 --warmup 1 --no-copy-ceiling --no-cpu-baseline $BENCH_ARGS) > "$OUT/prof_c$c.log" 2>&1 || { echo "prof failed"; tail -20 "$OUT/prof_c$c.log"; exit 4; }
    f=$(find "$OUT/prof_c$c" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/c${c}_kernel_stats.csv"
    python - "$OUT/c${c}_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print("   %-40s n=%-5s avg=%.3f ms" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
  fi
done
