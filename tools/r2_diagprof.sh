set -o pipefail
mkdir -p gpurun_out/diagprof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export ONEPASS_VARIANTS="#define TGPU_ONEPASS_NOLOOK;#define TGPU_ONEPASS_NOLOOK;#define TGPU_ONEPASS_NOEMIT;#define TGPU_ONEPASS_NOEMIT;#define TGPU_ONEPASS_NOLOOK
#define TGPU_ONEPASS_NOEMIT;#define TGPU_ONEPASS_NOLOOK
#define TGPU_ONEPASS_NOEMIT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/diagprof -o d -- python tools/onepass_diag.py 26 > gpurun_out/diagprof/d.log 2>&1; rc=$?; grep mode gpurun_out/diagprof/d.log; exit $rc
