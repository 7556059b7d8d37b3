#!/bin/bash
# The LDS-DMA settle: late-write counts and stuck calls of the speculation,
# and the configs' bench lines (decode/encode ms) with it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/c5_late_ab.sh "" "#define TGPU_NO_DMA_SETTLE 1" || exit 1
for c in 2 3 5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-copy-ceiling > gpurun_out/st_c$c.json 2>gpurun_out/st_c$c.err || { tail -5 gpurun_out/st_c$c.err; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/st_c$c.json')); r=d['roofline']; print('c$c value', d['value'], 'dec ms', r['avg_launch_ms'], 'frac', r['frac'], 'enc ms', r['encode']['avg_launch_ms'], 'enc frac', r['encode']['frac'])"
done
