#!/bin/bash
# SQ (shader) counters for the variable-length kernels: where the cycles of
# program_decode / program_write / index_tile_* go (issue vs wait vs LDS).
# Each pass is its own rocprofv3 run (--kernel-trace only, no tracing
# domains), 8 SQ counters at most per pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=$PWD/gpurun_out/${NAME:-sq}; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
PROG=${PROG:-"tools/kbench_prog.py --config 3 --dec 1,1,0 --rounds 1 --reps 1"}
P1="SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_LDS"
P2="SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_BRANCH"
i=0
for P in ${PASSES:-$P1 $P2}; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc ${P//,/ } --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- python3 "$OLDPWD"/$PROG) > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed $?"; tail -20 "$OUT/p$i.log"; exit 6; }
done
python3 tools/sq_summary.py "$OUT" > "$OUT/summary.txt" 2>&1
cat "$OUT/summary.txt"
