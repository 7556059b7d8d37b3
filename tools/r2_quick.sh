set -o pipefail
mkdir -p gpurun_out/q
for c in 2 3 4 5; do timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-copy-ceiling --no-cpu-baseline > gpurun_out/q/c$c.json 2>gpurun_out/q/c$c.err || exit 9; python -c "import json;d=json.loads(open('gpurun_out/q/c$c.json').read().strip().splitlines()[-1]);print($c, d['value'], d['ms_per_step'], d['roofline']['frac'])"; done
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling --irregular > gpurun_out/q/irregular.json 2>gpurun_out/q/irregular.err; rc=$?; grep "irregular.*ms" gpurun_out/q/irregular.err; exit $rc
