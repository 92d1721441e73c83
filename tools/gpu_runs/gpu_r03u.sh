# Round 3: the GEMV at the receive level (gfrx) at C3 (1,024 x 4 MiB) and C2
# with commit / receive 1 / 2, against the product; three repetitions.
set -o pipefail
O=gpurun_out/r03u; mkdir -p $O
R=$GRAFT_REPO_ROOT
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2"
for rep in 1 2 3; do
  for cv in "c3 --steps 20" "c2 --steps 60 --wave-prio 1,2"; do
    c=${cv%% *}; extra=${cv#* }
    for v in new gfrx; do
      lib=""; [ $v != new ] && lib=$R/ab/librbc_gpu_$v.so
      RBC_GPU_LIB_AB=$lib timeout -k 10 200 python bench.py $B --config $c $extra > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $c $v"; tail -20 $O/ab.err; exit 1; }
      python -c "import json; d=json.load(open('$O/ab.json')); print('$rep $c $extra $v', d['value'], {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','tree','verify','check','decode')})"
    done
  done
done
echo ok
