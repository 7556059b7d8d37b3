#!/bin/bash
# Parity subset for the program / index paths, then A/B timings of one
# schema-compiler define (VARS) on configs 3 and 4 and the config-5 call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=$PWD/gpurun_out/r2; mkdir -p "$OUT"
export TMPDIR=/tmp
if [[ -z $NOTEST ]]; then
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_index.py tests/test_unknown_tail.py tests/test_irregular_fixed.py tests/test_transcode.py} > "$OUT/pytest.log" 2>&1 \
  || { echo "tests failed $?"; tail -30 "$OUT/pytest.log"; exit 2; }
tail -1 "$OUT/pytest.log"
fi
for c in ${AB_CONFIGS:-3 4}; do
  timeout -k 10 400 python tools/kbench_jit.py --config $c --rounds 3 --var "" "$VARS" > "$OUT/kbench_c$c.log" 2>&1 || { echo "kbench c$c failed $?"; tail -20 "$OUT/kbench_c$c.log"; exit 3; }
  tail -2 "$OUT/kbench_c$c.log"
done
timeout -k 10 300 python tools/c5_time.py --sync-before --variants 1 > "$OUT/c5.log" 2>&1 || { echo "c5 failed $?"; tail -20 "$OUT/c5.log"; exit 4; }
tail -1 "$OUT/c5.log"
TGPU_JIT_DEFINES="$VARS" timeout -k 10 300 python tools/c5_time.py --sync-before --variants 1 > "$OUT/c5_var.log" 2>&1 || { echo "c5 var failed $?"; tail -20 "$OUT/c5_var.log"; exit 5; }
tail -1 "$OUT/c5_var.log"
echo done
