set -o pipefail
TESTS="tests/test_gpu_index.py tests/test_irregular_fixed.py tests/test_unknown_tail.py tests/test_shard_exchange.py tests/test_nested_containers.py tests/test_deep_skip.py" LOG=onepass LIMIT=800 bash tools/gpu_tests.sh || exit 1
bash tools/r2_quick.sh
