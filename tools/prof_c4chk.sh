set -o pipefail
mkdir -p gpurun_out/pc4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pc4 -o k -- python tools/c4chk.py > gpurun_out/pc4/log 2>&1; tail -6 gpurun_out/pc4/log
