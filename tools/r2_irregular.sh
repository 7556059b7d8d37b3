set -o pipefail
mkdir -p gpurun_out/r2
TESTS="tests/test_irregular_fixed.py tests/test_gpu_index.py tests/test_deep_skip.py" LOG=irregular LIMIT=500 bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling --irregular > gpurun_out/r2/irregular.json 2>gpurun_out/r2/irregular.err; rc=$?; cat gpurun_out/r2/irregular.err | grep irregular; exit $rc
