set -o pipefail
TESTS="tests/test_irregular_fixed.py tests/test_gpu_parity.py" LOG=stride2 LIMIT=600 bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling --irregular > gpurun_out/irr_s2.json 2>gpurun_out/irr_s2.err; rc=$?; grep "irregular.*ms" gpurun_out/irr_s2.err; exit $rc
