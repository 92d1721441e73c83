# Round 3: rbc_ctx_set_decode_priority in the product (bench default per
# config: GEMV at the receive level at N >= 128) -- the priority GPU test,
# then the default bench and every config against the committed library
# (ab/librbc_gpu_prev.so, the decode transforms at the commit level).
set -o pipefail
O=gpurun_out/r03v; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "priority or regen" > $O/parity.log 2>&1 || { echo PARITYFAIL; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 4"
for rep in 1 2; do
  for cv in "c2 --steps 150" "c1 --steps 60" "c3 --steps 20" "c4 --steps 40"; do
    c=${cv%% *}; extra=${cv#* }
    timeout -k 10 200 python bench.py $B --config $c $extra > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $c"; tail -20 $O/ab.err; exit 1; }
    python -c "import json; d=json.load(open('$O/ab.json')); print('$rep $c new', d['value'], d['config']['wave_priority'], {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','tree','verify','check','decode')})"
  done
done
echo ok
