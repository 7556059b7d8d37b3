set -o pipefail
mkdir -p gpurun_out/prof_c2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o c2 -- python bench.py --steps 5 --warmup 1 --no-copy-ceiling --no-cpu-baseline > gpurun_out/prof_c2/c2.json 2>gpurun_out/prof_c2/c2.err
