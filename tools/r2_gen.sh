set -o pipefail
TESTS="tests/test_nested_containers.py tests/test_gpu_parity.py tests/test_required.py tests/test_unions.py" LOG=gen LIMIT=700 bash tools/gpu_tests.sh || exit 1
timeout -k 10 400 python bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling --nested > gpurun_out/nested_bench.json 2> gpurun_out/nested_bench.err; rc=$?; python -c "import json;d=json.loads(open('gpurun_out/nested_bench.json').read().strip().splitlines()[-1]);n=d['nested'];print(n['encode_ms'], n['decode_ms'], n['roofline'])"; exit $rc
