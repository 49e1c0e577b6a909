set -e
mkdir -p gpurun_out/sw
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in "dna_j1:--opt probe_j=1" "dna_j2:--opt probe_j=2" "dna_j3:--opt probe_j=3" "dna_j4:--opt probe_j=4" "res_j2:--fq-residues 1 --opt probe_j=2"; do
  name=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sw/$name -o run -- python tools/bench_fq.py --pipeline 1 --reps 1 --n-reads 4000000 --no-cpu-baseline --handler-reads 0 $a > gpurun_out/sw/$name.json 2> gpurun_out/sw/$name.err
done
