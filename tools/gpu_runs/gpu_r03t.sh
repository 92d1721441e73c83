# Round 3: finer decode priority -- only the GEMV (gfrx) or only the FFT
# re-encode (fftrx) back at the receive level, against the product (both at
# the commit level), C2 / C1 / C4, three interleaved repetitions.
set -o pipefail
O=gpurun_out/r03t; mkdir -p $O
R=$GRAFT_REPO_ROOT
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2 --steps 60"
for rep in 1 2 3; do
  for c in c2 c1 c4; do
    for v in new gfrx fftrx; do
      lib=""; [ $v != new ] && lib=$R/ab/librbc_gpu_$v.so
      RBC_GPU_LIB_AB=$lib timeout -k 10 200 python bench.py $B --config $c > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $c $v"; tail -20 $O/ab.err; exit 1; }
      python -c "import json; d=json.load(open('$O/ab.json')); print('$rep $c $v', d['value'], {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','tree','verify','check','decode')})"
    done
  done
done
echo ok
