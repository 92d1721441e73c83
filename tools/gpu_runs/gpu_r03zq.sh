# Round 3: the Merkle build (one-wave tree blocks on the proposer stream) at
# issue level 3 (ab/librbc_gpu_tree3.so) against the commit level, C2 / C4 / C1.
set -o pipefail
O=gpurun_out/r03zq; mkdir -p $O
R=$GRAFT_REPO_ROOT
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2"
for rep in 1 2 3 4; do
  order="tree3 new"; [ $((rep % 2)) = 0 ] && order="new tree3"
  for c in c2 c4 c1; do
    for v in $order; do
      lib=""; [ $v != new ] && lib=$R/ab/librbc_gpu_$v.so
      RBC_GPU_LIB_AB=$lib timeout -k 10 200 python bench.py $B --config $c --steps 50 > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $c $v"; tail -20 $O/ab.err; exit 1; }
      python -c "import json; d=json.load(open('$O/ab.json')); print('$rep $c $v', d['value'], d['values_ok'], d['oracle_sample_ok'], {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','tree','verify','check','decode')})"
    done
  done
done
echo ok
