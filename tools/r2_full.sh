set -o pipefail
LOG=full LIMIT=1150 bash tools/gpu_tests.sh
