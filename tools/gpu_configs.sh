#!/bin/bash
# Configs 3 and 4 on one GPU: generator test, bench lines, rocprofv3 stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=$PWD/gpurun_out; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_bench_datagen.py -m gpu -x -q -p no:cacheprovider > "$OUT/pytest_gen.log" 2>&1 || { echo "gen test failed $?"; tail -30 "$OUT/pytest_gen.log"; exit 2; }
for c in ${CONFIGS:-3 4}; do
  timeout -k 10 600 python bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-copy-ceiling ${BENCH_ARGS:-} > "$OUT/bench_c$c.log" 2>&1 || { echo "bench c$c failed $?"; tail -30 "$OUT/bench_c$c.log"; exit 3; }
  tail -1 "$OUT/bench_c$c.log"
  if [[ -n $PROF ]]; then
    (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c$c" -o run -- python3 "$OLDPWD/bench.py" --config $c --steps 5 --warmup 1 --no-copy-ceiling) > "$OUT/prof_c$c.log" 2>&1 || { echo "prof c$c failed $?"; tail -20 "$OUT/prof_c$c.log"; exit 4; }
    head -8 "$OUT/prof_c$c/run_kernel_stats.csv" | cut -c1-220
  fi
done
echo done
