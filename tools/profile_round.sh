#!/bin/bash
# One round's measurement of the benched kernels, per workload (c2 c3 c4 c5
# nested): a rocprofv3 kernel-trace --stats pass, separate --pmc FETCH_SIZE and
# --pmc WRITE_SIZE passes (with the 1 GiB copy calibration of
# tools/pmc_calib.py once per call), and two SQ passes (8 SQ counters each).
# Every pass is its own rocprofv3 run with --kernel-trace only.
# tools/pmc_summary.py turns the FETCH/WRITE passes into pmc_<name>.json
# stamped with the kernel-source hash (tools/srchash.py) and GIT_COMMIT, which
# bench.py's roofline.traffic reads back (profiles/r<NN>/pmc/).
# usage: TAG=base NAMES="c2 c5" GIT_COMMIT=<sha> tools/profile_round.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$PWD
OUT=$ROOT/gpurun_out/prof/${TAG:-run}; mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_LDS"
P2="SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_BRANCH"
pass() {  # dir counters(or -) limit cmd...
  local d=$1 ctr=$2 lim=$3; shift 3
  local args="--kernel-trace --output-format csv"
  if [ "$ctr" = "-" ]; then args="$args --stats"; else args="--pmc ${ctr//,/ } $args"; fi
  echo "$(date +%T) $d" >> "$OUT/progress.log"
  (cd /tmp && timeout -s KILL "$lim" rocprofv3 $args -d "$d" -o run -- "$@") > "$d.log" 2>&1 \
    || { echo "pass $d failed $?"; tail -20 "$d.log"; exit 6; }
}
pass "$OUT/fetch_calib" FETCH_SIZE 120 python3 "$ROOT/tools/pmc_calib.py"
pass "$OUT/write_calib" WRITE_SIZE 120 python3 "$ROOT/tools/pmc_calib.py"
for name in ${NAMES:-c2 c3 c4 c5 nested}; do
  D=$OUT/$name; mkdir -p "$D"
  cp -r "$OUT/fetch_calib" "$OUT/write_calib" "$D/"
  case $name in
    nested) C=4; BENCH="$ROOT/bench.py --config 4 --records 65536 --steps 1 --warmup 1 --no-cpu-baseline --no-copy-ceiling --nested"; NFLAG=--nested ;;
    *) C=${name#c}; BENCH="$ROOT/bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --no-copy-ceiling"; NFLAG= ;;
  esac
  pass "$D/stats" - 240 python3 $BENCH
  pass "$D/fetch_bench" FETCH_SIZE 240 python3 $BENCH
  pass "$D/write_bench" WRITE_SIZE 240 python3 $BENCH
  pass "$D/p1" "$P1" 240 python3 $BENCH
  pass "$D/p2" "$P2" 240 python3 $BENCH
  python3 "$ROOT/tools/pmc_summary.py" "$D" --config $C $NFLAG --out "$D/pmc_$name.json" > "$D/summary.log" 2>&1 \
    || { cat "$D/summary.log"; exit 7; }
  python3 "$ROOT/tools/sq_summary.py" "$D" > "$D/sq.txt" 2>&1
  grep -h '"metric"' "$D/stats.log" > "$D/bench_line.json" || true
  rm -rf "$D/fetch_calib" "$D/write_calib"
  echo "== $name"; grep -A3 '_call"' "$D/pmc_$name.json" | head -20
done
echo done
