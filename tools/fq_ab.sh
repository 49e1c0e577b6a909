# same-box A/B of bench_fq configurations: tools/fq_ab.sh "name:args" ... (each run twice, alternating)
set -e
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for cfg in "$@"; do
    name=${cfg%%:*}; a=${cfg#*:}
    timeout -k 10 240 python -u tools/bench_fq.py --no-cpu-baseline --handler-reads 0 $a > gpurun_out/ab/${name}_$rep.json 2> gpurun_out/ab/${name}_$rep.err
  done
done
