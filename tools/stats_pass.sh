#!/bin/bash
# Reproducible per-config lines (round 6, verdict item 1): for each config,
# ONE run of `bench.py --config C` under `rocprofv3 --kernel-trace --stats`
# with BENCH_TRACE_MARKS=1 — the committed bench line and the committed
# kernel trace / stats come from the same process. tools/stats_check.py then
# cuts the trace into the K timed calls and compares the trace's call time
# with the line's HIP-event time (refused beyond 3 %).
# usage: CONFIGS="2 3 4 5" STEPS=20 TAG=final tools/stats_pass.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$PWD
OUT=$ROOT/gpurun_out/stats/${TAG:-run}; mkdir -p "$OUT"
export TMPDIR=/tmp BENCH_TRACE_MARKS=1
rc=0
for c in ${CONFIGS:-2 3 4 5}; do
  D=$OUT/c$c
  rm -rf "$D"; mkdir -p "$D"
  echo "$(date +%T) c$c" >> "$OUT/progress.log"
  (cd /tmp && timeout -k 10 ${LIMIT:-300} rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$D/prof" -o run -- python3 "$ROOT/bench.py" --config $c --steps ${STEPS:-20} \
     --warmup ${WARMUP:-3} --no-copy-ceiling ${BENCH_ARGS:---no-cpu-baseline}) \
     > "$D/line.json" 2> "$D/bench.err" || { echo "c$c failed $?"; tail -20 "$D/bench.err"; exit 5; }
  python3 "$ROOT/tools/stats_check.py" "$D/prof" "$D/line.json" --out "$D/check.json" > /dev/null
  r=$?; [ $r != 0 ] && rc=$r
  find "$D/prof" -name "*kernel_stats.csv" -exec cp {} "$D/kernel_stats.csv" \;
  python3 - "$D/check.json" <<'PY'
import json, sys
r = json.load(open(sys.argv[1]))
for s in ("decode", "encode"):
    x = r.get(s)
    if x:
        c = x.get("call", {})
        print("%s %s: events %.4f ms, trace span %s ms, kernels %.4f ms, frac events %.4f kernel %.4f agrees %s"
              % (r["config"][:9], s, x["event_ms"], c.get("span_ms"), x["kernel_ms"],
                 x["frac_events"], x["frac_kernel"], x["agrees"]))
PY
done
exit $rc
