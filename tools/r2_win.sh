set -o pipefail
TESTS="tests/test_gpu_parity.py tests/test_gpu_index.py tests/test_unknown_tail.py" LOG=win LIMIT=900 bash tools/gpu_tests.sh || exit 1
for c in 3 4 5; do timeout -k 10 300 python tools/kbench_jit.py --config $c --rounds 3 --var "" "#define TGPU_NO_WINCACHE" > gpurun_out/win_c$c.log 2>&1 || { tail -5 gpurun_out/win_c$c.log; exit 4; }; tail -2 gpurun_out/win_c$c.log; done
