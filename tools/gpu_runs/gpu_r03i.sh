# Round 3: gf_regen_kernel (interpolate's missing data rows: both waves of a
# block share one column tile, rows split between them) -- GPU parity first,
# then serial kernel stats at C4 / C2 and interleaved pipelined benches against
# the committed library (ab/librbc_gpu_r03base.so).
set -o pipefail
O=gpurun_out/r03i; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py > $O/parity.log 2>&1 || { echo PARITYFAIL; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
cd /tmp && export TMPDIR=/tmp
Q="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2"
for v in new base; do
  lib=""; [ $v != new ] && lib=$R/ab/librbc_gpu_r03$v.so
  for c in c4 c2 c1; do
    RBC_GPU_LIB_AB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/t_${c}_$v -o run --output-format csv -- python3 $R/bench.py --config $c --pipeline 0 --steps 5 --warmup 2 $Q > $R/$O/t_${c}_$v.json 2> $R/$O/t.log || { echo "TFAIL $v $c"; tail -5 $R/$O/t.log; exit 1; }
    grep -h "gf_short\|gf_rows\|gf_regen" $R/$O/t_${c}_$v/run_kernel_stats.csv | cut -d, -f1-4 | sed "s/^/$c $v /"
  done
done
cd $R
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2 --steps 60"
for rep in 1 2; do
  for c in c2 c4 c1; do
    for v in new base; do
      lib=""; [ $v != new ] && lib=$R/ab/librbc_gpu_r03$v.so
      RBC_GPU_LIB_AB=$lib timeout -k 10 200 python bench.py $B --config $c > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $c $v"; tail -20 $O/ab.err; exit 1; }
      python -c "import json; d=json.load(open('$O/ab.json')); print('$rep $c $v', d['value'], {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','verify','check','decode')})"
    done
  done
done
echo ok
