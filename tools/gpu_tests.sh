#!/bin/bash
# GPU pytest run: the selected tests first (TESTS, default: all -m gpu), one
# process, per-test timeout; log under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=$PWD/gpurun_out; mkdir -p "$OUT"
timeout -k 10 ${LIMIT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS:-} > "$OUT/${LOG:-pytest_gpu}.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/${LOG:-pytest_gpu}.log"; exit $rc
