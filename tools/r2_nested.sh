set -o pipefail
mkdir -p gpurun_out/r2
TESTS="tests/test_nested_containers.py tests/test_required.py tests/test_gpu_parity.py tests/test_irregular_fixed.py tests/test_gpu_index.py" LOG=nested LIMIT=700 bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling --irregular > gpurun_out/r2/irregular.json 2>gpurun_out/r2/irregular.err; rc=$?; grep irregular gpurun_out/r2/irregular.err; exit $rc
