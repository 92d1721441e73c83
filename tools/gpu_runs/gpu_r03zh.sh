# Round 3: C1 re-check of gf_regen_kernel's exact row counts against the
# committed build, order alternated per repetition (r03zg ran "new" first).
set -o pipefail
O=gpurun_out/r03zh; mkdir -p $O
R=$GRAFT_REPO_ROOT
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2"
for rep in 1 2 3 4; do
  order="old new"; [ $((rep % 2)) = 0 ] && order="new old"
  for c in c1 c2; do
    for v in $order; do
      lib=""; [ $v != new ] && lib=$R/ab/librbc_gpu_$v.so
      RBC_GPU_LIB_AB=$lib timeout -k 10 200 python bench.py $B --config $c --steps 60 > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $c $v"; tail -20 $O/ab.err; exit 1; }
      python -c "import json; d=json.load(open('$O/ab.json')); print('$rep $c $v', d['value'], {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','tree','verify','check','decode')})"
    done
  done
done
echo ok
