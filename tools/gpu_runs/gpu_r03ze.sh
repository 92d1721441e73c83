# Round 3: the leaf hashing (sha_rows_kernel) in 64- / 128-thread blocks (A/B builds)
# against the product (256-thread blocks), C4 / C2 / C1, 3 reps.
set -o pipefail
O=gpurun_out/r03ze; mkdir -p $O
R=$GRAFT_REPO_ROOT
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2"
for rep in 1 2 3; do
  for cv in "c4 --steps 40" "c2 --steps 100" "c1 --steps 60"; do
    c=${cv%% *}; extra=${cv#* }
    for v in new rows64 rows128; do
      lib=""; [ $v != new ] && lib=$R/ab/librbc_gpu_$v.so
      RBC_GPU_LIB_AB=$lib timeout -k 10 200 python bench.py $B --config $c $extra > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $c $v"; tail -20 $O/ab.err; exit 1; }
      python -c "import json; d=json.load(open('$O/ab.json')); print('$rep $c $v', d['value'], {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','tree','verify','check','decode')})"
    done
  done
done
echo ok
