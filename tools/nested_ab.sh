#!/bin/bash
# Nested leg A/B (bench line only): "name:ENV=V,ENV=V" variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/nab
DEF="default: rt0_80k:TGPU_NESTED_RTILE=0 rt0_53k:TGPU_NESTED_RTILE=0,TGPU_NESTED_LDS=54613"
for spec in ${VARIANTS:-$DEF}; do
  name=${spec%%:*}; envs=${spec#*:}
  (
    IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
    timeout -k 10 300 python3 bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline --no-copy-ceiling --nested > gpurun_out/nab/$name.json 2> gpurun_out/nab/$name.err
  ) || { echo "fail $name"; tail -5 gpurun_out/nab/$name.err; exit 2; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); n=d['nested']; print(sys.argv[2], 'enc', n['encode_ms'], 'dec', n['decode_ms'])" gpurun_out/nab/$name.json $name
done
