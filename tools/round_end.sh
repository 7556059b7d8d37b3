#!/bin/bash
# Round-end measurement on one GPU: smoke, the default bench line (config 2
# with CPU baseline and copy ceiling), its rocprofv3 kernel stats, configs 1
# and 3-5 bench lines (3/4 with host-start and host-batch, 3-5 with
# transcoding), config 2's host-start rates, the irregular-stream and
# nested-container legs, skim (configs 2-4) and transcoding (configs 2-4).
# Outputs under gpurun_out/final/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=$PWD/gpurun_out/final; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed $?"; tail -20 "$OUT/smoke.log"; exit 2; }
timeout -k 10 600 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { echo "bench failed $?"; tail -20 "$OUT/bench_default.err"; exit 3; }
cat "$OUT/bench_default.json"
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_default" -o run -- python3 "$OLDPWD/bench.py" --steps 5 --warmup 1 --no-copy-ceiling --no-cpu-baseline) > "$OUT/prof_default.log" 2>&1 || { echo "prof failed $?"; tail -20 "$OUT/prof_default.log"; exit 4; }
timeout -k 10 300 python bench.py --config 1 > "$OUT/bench_c1.json" 2> "$OUT/bench_c1.err" || { echo "bench c1 failed $?"; exit 5; }
timeout -k 10 400 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-copy-ceiling --host-start > "$OUT/bench_c2_host_start.json" 2> "$OUT/bench_c2_host_start.err" || { echo "host-start c2 failed $?"; exit 5; }
for c in ${CONFIGS:-3 4 5}; do
  EXTRA="--transcode"; [ $c != 5 ] && EXTRA="$EXTRA --host-start --host-batch --skim"
  timeout -k 10 600 python bench.py --config $c --steps 10 --warmup 2 --no-copy-ceiling $EXTRA > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err" || { echo "bench c$c failed $?"; tail -20 "$OUT/bench_c$c.err"; exit 5; }
  tail -c 300 "$OUT/bench_c$c.json"
done
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling --skim --transcode > "$OUT/bench_c2_skim.json" 2> "$OUT/bench_c2_skim.err" || { echo "skim c2 failed $?"; exit 6; }
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling --irregular > "$OUT/bench_irregular.json" 2> "$OUT/bench_irregular.err" || { echo "irregular failed $?"; exit 6; }
timeout -k 10 400 python bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling --nested > "$OUT/bench_nested.json" 2> "$OUT/bench_nested.err" || { echo "nested failed $?"; exit 7; }
echo done
