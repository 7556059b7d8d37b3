# Nested-leg check: the general-reader GPU tests, then the nested profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_nested_containers.py tests/test_deep_skip.py tests/test_unknown_tail.py tests/test_gpu_parity.py tests/test_compact_v1.py tests/test_oracle_semantics.py > gpurun_out/nested_tests.log 2>&1 && bash tools/prof_nested.sh
