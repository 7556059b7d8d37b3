set -o pipefail
TESTS="tests/test_gpu_index.py" PYTEST_ARGS="-k onepass" LOG=onepass2 LIMIT=300 bash tools/gpu_tests.sh || exit 1
timeout -k 10 400 python tools/kbench_jit.py --config 5 --rounds 3 --var "" "#define TGPU_KOVER 1024" "#define TGPU_KOVER 512" > gpurun_out/kov.log 2>&1; rc=$?; tail -4 gpurun_out/kov.log; [ $rc = 0 ] || exit $rc
TGPU_INDEX_ONEPASS=1 timeout -k 10 400 python tools/kbench_jit.py --config 5 --rounds 3 --var "" "#define TGPU_KOVER 1024" "#define TGPU_REC_TILE 8192" "#define TGPU_KOVER 1024
#define TGPU_REC_TILE 8192" > gpurun_out/kov1.log 2>&1; rc=$?; tail -5 gpurun_out/kov1.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling --nested > gpurun_out/nested_bench.json 2> gpurun_out/nested_bench.err; rc=$?; tail -3 gpurun_out/nested_bench.err; python -c "import json;d=json.loads(open('gpurun_out/nested_bench.json').read().strip().splitlines()[-1]);print(json.dumps(d['nested']))"; exit $rc
