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
echo done
