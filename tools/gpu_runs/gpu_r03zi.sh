# Round 3: the W = 3 gf_regen form (16 rows a wave, 3 waves) at C1 and C2 too
# (ab/librbc_gpu_w3.so) against the product (W = 4, 12 rows a wave, 2 waves).
set -o pipefail
O=gpurun_out/r03zi; mkdir -p $O
R=$GRAFT_REPO_ROOT
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2"
for rep in 1 2 3 4; do
  order="w3 new"; [ $((rep % 2)) = 0 ] && order="new w3"
  for c in c1 c2; do
    for v in $order; do
      lib=""; [ $v != new ] && lib=$R/ab/librbc_gpu_$v.so
      RBC_GPU_LIB_AB=$lib timeout -k 10 200 python bench.py $B --config $c --steps 60 > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $c $v"; tail -20 $O/ab.err; exit 1; }
      python -c "import json; d=json.load(open('$O/ab.json')); print('$rep $c $v', d['value'], {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','tree','verify','check','decode')})"
    done
  done
done
echo ok
