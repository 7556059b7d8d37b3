set -o pipefail
mkdir -p gpurun_out/prof_c4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 -- python bench.py --config 4 --steps 5 --warmup 1 --no-copy-ceiling --no-cpu-baseline > gpurun_out/prof_c4/c4.json 2>gpurun_out/prof_c4/c4.err
