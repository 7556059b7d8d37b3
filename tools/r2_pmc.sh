set -o pipefail
for c in 5 3 4; do CONFIG=$c bash tools/pmc_config.sh > gpurun_out/pmc_c$c.out 2>&1 || { tail -30 gpurun_out/pmc_c$c.out; exit 5; }; tail -3 gpurun_out/pmc_c$c.out; done
