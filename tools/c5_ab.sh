#!/bin/bash
# Config-5 index work on one GPU: index parity tests, then bench lines with
# the stored-starts index (default) and without (TGPU_INDEX_STARTS=0), the
# branchy-walk A/B through the schema compiler, and rocprofv3 kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=$PWD/gpurun_out/c5ab; mkdir -p "$OUT"
export TMPDIR=/tmp
if [[ -z $NOTEST ]]; then
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_index.py tests/test_unknown_tail.py tests/test_irregular_fixed.py ${TESTS:-} > "$OUT/pytest.log" 2>&1 \
  || { echo "tests failed $?"; tail -30 "$OUT/pytest.log"; exit 2; }
tail -2 "$OUT/pytest.log"
fi
B="bench.py --config ${CONFIG:-5} --steps 10 --warmup 2 --no-cpu-baseline --no-copy-ceiling"
timeout -k 10 300 python $B > "$OUT/bench_starts.json" 2> "$OUT/bench_starts.err" || { echo "bench failed $?"; tail -20 "$OUT/bench_starts.err"; exit 3; }
python3 -c "import json;d=json.loads(open('$OUT/bench_starts.json').read().strip().splitlines()[-1]);r=d['roofline'];print('starts',d['value'],r['avg_launch_ms'],r['frac'])"
TGPU_INDEX_STARTS=0 timeout -k 10 300 python $B > "$OUT/bench_fused.json" 2> "$OUT/bench_fused.err" || { echo "bench fused failed $?"; tail -20 "$OUT/bench_fused.err"; exit 4; }
python3 -c "import json;d=json.loads(open('$OUT/bench_fused.json').read().strip().splitlines()[-1]);r=d['roofline'];print('fused',d['value'],r['avg_launch_ms'],r['frac'])"
if [[ -n $VARS ]]; then
  timeout -k 10 400 python tools/kbench_jit.py --config ${CONFIG:-5} --rounds 3 --var "" "$VARS" > "$OUT/kbench.log" 2>&1 || { echo "kbench failed $?"; tail -20 "$OUT/kbench.log"; exit 5; }
  cat "$OUT/kbench.log" | tail -3
fi
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$OLDPWD/bench.py" --config ${CONFIG:-5} --steps 5 --warmup 1 --no-cpu-baseline --no-copy-ceiling) > "$OUT/prof.log" 2>&1 || { echo "prof failed $?"; tail -20 "$OUT/prof.log"; exit 6; }
python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')))[:14]:
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6, 4))"
for c in ${EXTRA_CONFIGS:-}; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-copy-ceiling > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err" || { echo "bench c$c failed $?"; tail -20 "$OUT/bench_c$c.err"; exit 7; }
  python3 -c "import json;d=json.loads(open('$OUT/bench_c$c.json').read().strip().splitlines()[-1]);r=d['roofline'];print('c$c',d['value'],r['avg_launch_ms'],r['frac'],r['encode']['avg_launch_ms'])"
done
echo done
