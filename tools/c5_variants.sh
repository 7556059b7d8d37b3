cd $GRAFT_REPO_ROOT
for v in "" "#define TGPU_KOVER 1024" "#define TGPU_KOVER 512" "#define TGPU_KOVER 2048"; do
  TGPU_JIT_DEFINES="$v" timeout -k 10 200 python tools/c5_time.py --sync-before --variants 1 --reps 6 > gpurun_out/c5v.log 2>&1 || { echo "failed $?"; tail -5 gpurun_out/c5v.log; exit 2; }
  echo "$v: $(tail -1 gpurun_out/c5v.log)"
done
