# Round 3: GF kernel A/B on one box (previous kernels vs the scalar-offset /
# double-buffered ones): serial kernel traces at C4 and C2, interleaved
# pipelined benches; then the rocprof evidence of the default (profile.sh r03).
set -o pipefail
O=gpurun_out/r03e; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
Q="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2"
for rep in 1 2; do
for v in base oldgf; do
  lib=""; [ $v != base ] && lib=$R/ab/librbc_gpu_$v.so
  for c in c4 c2; do
    RBC_GPU_LIB_AB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/t_${c}_${v}_$rep -o run --output-format csv -- python3 $R/bench.py --config $c --pipeline 0 --steps 5 --warmup 2 $Q > $R/$O/t_${c}_${v}_$rep.json 2> $R/$O/t.log || { echo "TFAIL $v $c"; exit 1; }
    grep -h "gf_short\|gf_rows" $R/$O/t_${c}_${v}_$rep/run_kernel_stats.csv | cut -d, -f1-4 | sed "s/^/$rep $c $v /"
  done
done
done
cd $R
B="--no-cpu-baseline --no-pcie --steps 60"
run() {  # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py $B "$@" > $O/$tag.json 2>> $O/runs.err || { echo "RUNFAIL $tag"; tail -20 $O/runs.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['ms_per_step'], {k: round(v, 3) for k, v in d['stage_ms'].items()})"
}
for rep in 1 2; do
  for c in c2 c4; do
    run ${c}_base_$rep --config $c
    RBC_GPU_LIB_AB=$R/ab/librbc_gpu_oldgf.so run ${c}_oldgf_$rep --config $c
  done
done
timeout -k 10 900 bash tools/profile.sh r03 > $O/profile.log 2>&1 || { echo PROFFAIL; tail -30 $O/profile.log; exit 1; }
echo ok
