# Round 3, final code: shard row pitch alignment (--shard-align 64 / 128 / 256
# bytes) at C2, three repetitions.
set -o pipefail
O=gpurun_out/r03zs; mkdir -p $O
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2 --steps 100"
for rep in 1 2 3; do
  for al in 64 128 256 512; do
    timeout -k 10 200 python bench.py $B --shard-align $al > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $al"; tail -20 $O/ab.err; exit 1; }
    python -c "import json; d=json.load(open('$O/ab.json')); print('$rep c2 align $al', d['value'], d['values_ok'], {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','tree','verify','check','decode')})"
  done
done
echo ok
