#!/bin/bash
# nested leg A/B: default, then TGPU_NESTED_LDS variants (bench line only)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/nab
for v in 81920 65536 163840; do
  TGPU_NESTED_LDS=$v timeout -k 10 300 python3 bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline --no-copy-ceiling --nested > gpurun_out/nab/lds_$v.json 2> gpurun_out/nab/lds_$v.err || { echo "fail $v"; tail -5 gpurun_out/nab/lds_$v.err; exit 2; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); n=d['nested']; print(sys.argv[2], 'enc', n['encode_ms'], 'dec', n['decode_ms'])" gpurun_out/nab/lds_$v.json $v
done
