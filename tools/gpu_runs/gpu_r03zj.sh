# Round 3: four shard sets in flight (--sets 4: the proposer may commit one
# batch further ahead, so its encode can fill the receiver's FFT tail)
# against three, C2 / C1 / C4, order alternated per repetition.
set -o pipefail
O=gpurun_out/r03zj; mkdir -p $O
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2"
for rep in 1 2 3; do
  order="3 4"; [ $((rep % 2)) = 0 ] && order="4 3"
  for cv in "c2 --steps 100" "c1 --steps 60" "c4 --steps 40"; do
    c=${cv%% *}; extra=${cv#* }
    for v in $order; do
      timeout -k 10 200 python bench.py $B --config $c $extra --sets $v > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $c $v"; tail -20 $O/ab.err; exit 1; }
      python -c "import json; d=json.load(open('$O/ab.json')); print('$rep $c sets=$v', d['value'], d['values_ok'], {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','tree','verify','check','decode')})"
    done
  done
done
echo ok
