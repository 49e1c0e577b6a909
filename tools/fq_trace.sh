# kernel traces of bench_fq configurations (pipeline 1, 4M reads): tools/fq_trace.sh "name:args" ...
set -e
mkdir -p gpurun_out/tr
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in "$@"; do
  name=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr/$name -o run -- python tools/bench_fq.py --pipeline 1 --reps 1 --n-reads 4000000 --no-cpu-baseline --handler-reads 0 $a > gpurun_out/tr/$name.json 2> gpurun_out/tr/$name.err
done
