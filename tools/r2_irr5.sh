set -o pipefail
TESTS="tests/test_irregular_fixed.py tests/test_unknown_tail.py" LOG=irr5 LIMIT=600 bash tools/gpu_tests.sh || exit 1
bash tools/r2_quick.sh
