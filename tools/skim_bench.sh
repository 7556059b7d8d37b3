#!/bin/bash
# Skim (tgpu_skim_batch) rates on configs 2-4 plus rocprofv3 kernel stats of
# the config-3 run. Outputs under gpurun_out/skim/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=$PWD/gpurun_out/skim; mkdir -p "$OUT"
export TMPDIR=/tmp
for c in ${CONFIGS:-2 3 4}; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-copy-ceiling --no-cpu-baseline --skim > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err" || { echo "bench c$c failed $?"; tail -20 "$OUT/bench_c$c.err"; exit 5; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_c$c.json')); print($c, d['skim'])"
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c3" -o run -- python3 "$OLDPWD/bench.py" --config 3 --steps 2 --warmup 1 --no-copy-ceiling --skim) > "$OUT/prof_c3.log" 2>&1 || { echo "prof failed $?"; tail -20 "$OUT/prof_c3.log"; exit 4; }
echo done
