#!/bin/bash
# PMC FETCH_SIZE / WRITE_SIZE of one config's bench under schema-compiler
# variants (TGPU_JIT_DEFINES) or environment switches, each its own
# rocprofv3 --kernel-trace run (round 6: config 4 decode traffic A/B).
# usage: CONFIG=4 tools/pmc_variants.sh "" "#define TGPU_RR_STORE16" "env:TGPU_ARENA_PACK=0"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$PWD
OUT=$ROOT/gpurun_out/pmcvar/${TAG:-run}; mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for v in "$@"; do
  D=$OUT/v$i; mkdir -p "$D"; echo "$v" > "$D/variant.txt"
  unset TGPU_JIT_DEFINES
  ENVV=""
  case "$v" in
    env:*) ENVV="${v#env:}" ;;
    "") ;;
    *) export TGPU_JIT_DEFINES="$v" ;;
  esac
  for ctr in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && env $ENVV timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace --output-format csv \
       -d "$D/$ctr" -o run -- python3 "$ROOT/bench.py" --config ${CONFIG:-4} --steps 2 --warmup 1 \
       --no-cpu-baseline --no-copy-ceiling) > "$D/$ctr.log" 2>&1 || { echo "v$i $ctr failed"; tail -5 "$D/$ctr.log"; exit 6; }
  done
  i=$((i+1))
done
echo done
