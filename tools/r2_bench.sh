set -o pipefail
nproc; python -c "import os; print('aff', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>&1; ls profiles | head -3
python -c "import bench; print('pmc', bench.pmc_traffic('plan_binary_decode_kernel', 1<<26, 2))"
mkdir -p gpurun_out/r2
timeout -k 10 300 python bench.py --config 1 > gpurun_out/r2/c1.json 2>gpurun_out/r2/c1.err && tail -1 gpurun_out/r2/c1.json
timeout -k 10 400 python bench.py > gpurun_out/r2/c2.json 2>gpurun_out/r2/c2.err && tail -1 gpurun_out/r2/c2.json
for c in 3 4 5; do timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 2 --no-copy-ceiling > gpurun_out/r2/c$c.json 2>gpurun_out/r2/c$c.err || exit 9; tail -1 gpurun_out/r2/c$c.json; done
