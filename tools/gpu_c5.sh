#!/bin/bash
# Config-5 check on one GPU: the index tests, a config-5 bench line, its
# rocprofv3 kernel stats and the index phase timings. Outputs under
# gpurun_out/c5/ (TAG names the run).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=$PWD/gpurun_out/c5${TAG:+_$TAG}; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_index.py tests/test_index_repairs.py} -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/pytest.log"; exit 2; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline --no-copy-ceiling > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 3; }
python -c "import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']; print('value', d['value'], 'dec ms', r['avg_launch_ms'], 'frac', r['frac'], 'enc ms', r['encode']['avg_launch_ms'], 'enc frac', r['encode']['frac'])"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$OLDPWD/bench.py" --config 5 --steps 5 --warmup 1 --no-copy-ceiling --no-cpu-baseline) > "$OUT/prof.log" 2>&1 || { echo "prof failed"; tail -20 "$OUT/prof.log"; exit 4; }
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats.csv"
python - "$OUT/kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print("%-40s n=%-5s avg=%.3f ms" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
TGPU_INDEX_TIMING=2 timeout -k 10 300 python tools/c5_time.py --records 67108864 --variants 1 --reps 3 > "$OUT/phases.log" 2>&1 || { echo "phases failed"; tail -20 "$OUT/phases.log"; exit 5; }
tail -25 "$OUT/phases.log"
