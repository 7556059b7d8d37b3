set -o pipefail
mkdir -p gpurun_out/pn
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pn -o n -- python bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline --no-copy-ceiling --nested > gpurun_out/pn/out.json 2> gpurun_out/pn/err
