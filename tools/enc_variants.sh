#!/bin/bash
# Plan encode tile variants (TGPU_PLAN_ENCODE="T,nt") on config 2: encode ms per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=$PWD/gpurun_out/encvar; mkdir -p "$OUT"
for v in ${VARIANTS:-512,1 512,1,1 256,1,1 256,1}; do
  TGPU_PLAN_ENCODE=$v timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-copy-ceiling > "$OUT/b_$v.json" 2> "$OUT/b_$v.err" || { echo "variant $v failed"; tail -5 "$OUT/b_$v.err"; exit 2; }
  python -c "import json,sys; d=json.load(open('$OUT/b_$v.json')); r=d['roofline']; print('$v', 'value', d['value'], 'dec', r['avg_launch_ms'], 'enc', r['encode']['avg_launch_ms'], r['encode']['frac'])"
done
