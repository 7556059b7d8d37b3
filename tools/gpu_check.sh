#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Stops at the first step that crashes/times out (exit >= 2 for pytest,
# != 0 otherwise); writes logs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=$PWD/gpurun_out
mkdir -p "$OUT"
STEPS=${STEPS:-all}
run() { echo "== $*" >&2; }

if [[ $STEPS == all || $STEPS == *test* ]]; then
  run pytest
  timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
  if [[ $rc -ge 2 ]]; then exit $rc; fi
fi
if [[ $STEPS == all || $STEPS == *smoke* ]]; then
  run smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed $?"; tail -20 "$OUT/smoke.log"; exit 3; }
  tail -2 "$OUT/smoke.log"
fi
if [[ $STEPS == all || $STEPS == *bench* ]]; then
  run bench
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1 || { echo "bench failed $?"; tail -20 "$OUT/bench.log"; exit 4; }
  tail -1 "$OUT/bench.log"
fi
if [[ $STEPS == all || $STEPS == *prof* ]]; then
  run rocprof
  export TMPDIR=/tmp
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$OLDPWD/bench.py" --steps 5 --warmup 1 --no-cpu-baseline ${PROF_ARGS:-}) > "$OUT/prof.log" 2>&1 || { echo "rocprof failed $?"; tail -20 "$OUT/prof.log"; exit 5; }
  find "$OUT/prof" -name "*stats*" | head
fi
if [[ $STEPS == *pmc* ]]; then
  run pmc
  export TMPDIR=/tmp
  P=$OUT/pmc; rm -rf "$P"; mkdir -p "$P"
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$(echo ${c%_SIZE} | tr A-Z a-z)
    (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$P/${d}_calib" -o run -- python3 "$OLDPWD/tools/pmc_calib.py") > "$P/${d}_calib.log" 2>&1 || { echo "pmc calib $c failed $?"; tail -20 "$P/${d}_calib.log"; exit 6; }
    (cd /tmp && timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$P/${d}_bench" -o run -- python3 "$OLDPWD/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-copy-ceiling ${PROF_ARGS:-}) > "$P/${d}_bench.log" 2>&1 || { echo "pmc bench $c failed $?"; tail -20 "$P/${d}_bench.log"; exit 6; }
  done
  python3 tools/pmc_summary.py "$P" ${PMC_RECORDS:-67108864} "$OUT/pmc_latest.json" > "$P/summary.log" 2>&1 || { echo "pmc summary failed"; tail -20 "$P/summary.log"; }
  tail -30 "$P/summary.log"
fi
echo done
