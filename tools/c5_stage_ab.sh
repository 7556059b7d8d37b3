for v in "#define TGPU_SPEC_CHECK 1" "#define TGPU_SPEC_CHECK 1
#define TGPU_SPEC_REGSTAGE 1"; do
  TGPU_INDEX_TIMING=2 TGPU_JIT_DEFINES="$v" timeout -k 10 200 python tools/c5_time.py --variants 1 --reps 16 --stats > gpurun_out/c5ab.log 2>&1 || exit 1
  echo "== $v" | tr '\n' ' '; echo
  grep -E "spec check" gpurun_out/c5ab.log | awk '{s+=$(NF-8)+0; if ($(NF-8)+0>0) n++} END {print "stuck tiles total", s, "calls with stuck", n, "of", NR}'
  grep "decode wall" gpurun_out/c5ab.log
done
