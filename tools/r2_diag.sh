set -o pipefail
mkdir -p gpurun_out/diag
timeout -k 10 200 python tools/onepass_diag.py 22 > gpurun_out/diag/d22.log 2>&1; rc=$?; tail -8 gpurun_out/diag/d22.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/onepass_diag.py 26 > gpurun_out/diag/d26.log 2>&1; rc=$?; tail -8 gpurun_out/diag/d26.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/onepass_diag.py 26 stats > gpurun_out/diag/d26s.log 2>&1; rc=$?; tail -12 gpurun_out/diag/d26s.log; exit $rc
