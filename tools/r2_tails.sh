timeout -k 10 300 python tools/kbench_jit.py --config 4 --rounds 3 --var "" "#define TGPU_NO_TAILS" > gpurun_out/tails_c4.log 2>&1; tail -2 gpurun_out/tails_c4.log
TGPU_JIT=0 timeout -k 10 200 python tools/c4chk.py 2>/dev/null | tail -5 | sed 's/^/interp /'
