set -u
R=$(pwd)
for C in ${CONFIGS:-C3 C5}; do
  c=$(echo $C | tr A-Z a-z)
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$c -o run -- python3 $R/bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline) > $R/gpurun_out/prof_$c.log 2>&1 || exit 1
  CONFIG=$C PMC_OUT=$R/gpurun_out/pmc_$c bash tools/pmc.sh || exit 1
done
