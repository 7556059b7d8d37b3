set -o pipefail
for k in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline --no-copy-ceiling > gpurun_out/c2_$k.json 2>/dev/null || exit 3; python -c "import json;d=json.loads(open('gpurun_out/c2_$k.json').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['avg_launch_ms'], d['roofline']['encode']['avg_launch_ms'])"; done
