set -o pipefail
mkdir -p gpurun_out/prof_irr2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_irr2 -o irr -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-copy-ceiling --irregular > gpurun_out/prof_irr2/irr.json 2>gpurun_out/prof_irr2/irr.err
