# Round 3: shared-path ECHO verify (sha_rx leaf hashing + merkle_path_kernel,
# ab/librbc_gpu_path.so) at C1 / C2, where the product walks each branch in sha_rx.
set -o pipefail
O=gpurun_out/r03zl; mkdir -p $O
R=$GRAFT_REPO_ROOT
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2"
for rep in 1 2 3 4; do
  order="path new"; [ $((rep % 2)) = 0 ] && order="new path"
  for c in c1 c2; do
    for v in $order; do
      lib=""; [ $v != new ] && lib=$R/ab/librbc_gpu_$v.so
      RBC_GPU_LIB_AB=$lib timeout -k 10 200 python bench.py $B --config $c --steps 60 > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $c $v"; tail -20 $O/ab.err; exit 1; }
      python -c "import json; d=json.load(open('$O/ab.json')); print('$rep $c $v', d['value'], d['values_ok'], d['oracle_sample_ok'], {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','tree','verify','check','decode')})"
    done
  done
done
echo ok
