#!/bin/bash
# Round-end measurement on one GPU: smoke, the default bench line (config 2
# with CPU baseline and copy ceiling), its rocprofv3 kernel stats, and
# configs 3-5 bench lines with transcoding. Outputs under gpurun_out/final/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=$PWD/gpurun_out/final; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed $?"; tail -20 "$OUT/smoke.log"; exit 2; }
timeout -k 10 600 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { echo "bench failed $?"; tail -20 "$OUT/bench_default.err"; exit 3; }
cat "$OUT/bench_default.json"
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_default" -o run -- python3 "$OLDPWD/bench.py" --steps 5 --warmup 1 --no-copy-ceiling --no-cpu-baseline) > "$OUT/prof_default.log" 2>&1 || { echo "prof failed $?"; tail -20 "$OUT/prof_default.log"; exit 4; }
for c in ${CONFIGS:-3 4 5}; do
  timeout -k 10 600 python bench.py --config $c --steps 10 --warmup 2 --no-copy-ceiling --transcode > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err" || { echo "bench c$c failed $?"; tail -20 "$OUT/bench_c$c.err"; exit 5; }
done
echo done
