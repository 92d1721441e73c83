# Round 3: per-config decode levels (bench default) against both transforms at
# the commit level (--decode-prio c,c), same library, interleaved, 3 reps.
set -o pipefail
O=gpurun_out/r03w; mkdir -p $O
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2"
for rep in 1 2 3; do
  for cv in "c2 --steps 150" "c3 --steps 20" "c1 --steps 60"; do
    c=${cv%% *}; extra=${cv#* }
    for dp in default c,c r,c; do
      a=""; [ $dp != default ] && a="--decode-prio $dp"
      timeout -k 10 200 python bench.py $B --config $c $extra $a > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $c"; tail -20 $O/ab.err; exit 1; }
      python -c "import json; d=json.load(open('$O/ab.json')); w=d['config']['wave_priority']; print('$rep $c $dp', d['value'], (w['decode_gemv'], w['decode_reencode']), {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','tree','verify','check','decode')})"
    done
  done
done
echo ok
