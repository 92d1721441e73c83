# Round 3: C1 (N = 64: one leaf wave per SIMD, a 745-compression chain per
# lane, on the proposer stream that sets C1's step) under other commit /
# receive issue levels than the default 0 / 2; two repetitions.
set -o pipefail
O=gpurun_out/r03zn; mkdir -p $O
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2 --config c1 --steps 60"
for rep in 1 2; do
  for wp in 0,2 2,0 0,0 1,0 3,2; do
    timeout -k 10 200 python bench.py $B --wave-prio $wp > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $wp"; tail -20 $O/ab.err; exit 1; }
    python -c "import json; d=json.load(open('$O/ab.json')); print('$rep c1 $wp', d['value'], {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','tree','verify','check','decode')})"
  done
done
echo ok
