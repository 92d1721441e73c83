# Round 3: gf_regen_kernel with exact per-wave row counts (no 4-row groups)
# against the committed build (ab/librbc_gpu_old.so): GPU parity of the new
# build, then C2 / C1 / C4 interleaved, 3 reps.
set -o pipefail
O=gpurun_out/r03zg; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py > $O/parity.log 2>&1 || { echo PARITYFAIL; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2"
for rep in 1 2 3; do
  for cv in "c2 --steps 100" "c1 --steps 60" "c4 --steps 40"; do
    c=${cv%% *}; extra=${cv#* }
    for v in new old; do
      lib=""; [ $v != new ] && lib=$R/ab/librbc_gpu_$v.so
      RBC_GPU_LIB_AB=$lib timeout -k 10 200 python bench.py $B --config $c $extra > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $c $v"; tail -20 $O/ab.err; exit 1; }
      python -c "import json; d=json.load(open('$O/ab.json')); print('$rep $c $v', d['value'], {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','tree','verify','check','decode')})"
    done
  done
done
echo ok
