#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE) and SQ counters of one bench config's
# kernels: each counter set is its own rocprofv3 --pmc run (kernel trace only,
# no tracing domains; <= 8 SQ / 4 TCC counters per pass), plus the copy
# calibration (tools/pmc_calib.py) in the FETCH/WRITE passes. Then
# tools/pmc_summary.py writes profiles/pmc_c$CONFIG.json and
# tools/sq_summary.py the SQ table. usage: CONFIG=5 tools/pmc_config.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
C=${CONFIG:-5}
OUT=$PWD/gpurun_out/pmc_c$C; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="$PWD/bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --no-copy-ceiling"
run() {  # name counters cmd...
  local name=$1 ctr=$2; shift 2
  (cd /tmp && timeout -s KILL 170 rocprofv3 --pmc ${ctr//,/ } --kernel-trace --output-format csv -d "$OUT/$name" -o run -- "$@") > "$OUT/$name.log" 2>&1 || { echo "pass $name failed $?"; tail -20 "$OUT/$name.log"; exit 6; }
}
run fetch_calib FETCH_SIZE python3 "$PWD/tools/pmc_calib.py"
run write_calib WRITE_SIZE python3 "$PWD/tools/pmc_calib.py"
run fetch_bench FETCH_SIZE python3 $BENCH
run write_bench WRITE_SIZE python3 $BENCH
tail -1 "$OUT/fetch_bench.log" > "$OUT/bench_line.json" || true
python3 tools/pmc_summary.py "$OUT" --config $C > "$OUT/summary.log" 2>&1 || { cat "$OUT/summary.log"; exit 7; }
P1="SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_LDS"
P2="SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_BRANCH"
run p1 "$P1" python3 $BENCH
run p2 "$P2" python3 $BENCH
python3 tools/sq_summary.py "$OUT" > "$OUT/sq.txt" 2>&1
cat "$OUT/summary.log" | tail -40
