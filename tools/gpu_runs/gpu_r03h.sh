# Round 3: wave-priority A/B under the pipelined schedule (VERDICT r02 item 4:
# re-balance the streams now that the proposer is critical at C2, while at C4
# the receiver is), two interleaved repetitions per setting, C2 and C4.
set -o pipefail
O=gpurun_out/r03h; mkdir -p $O
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2 --steps 60"
for rep in 1 2; do
  for c in c2 c4; do
    for p in 0,2 0,0 0,1 0,3 1,2 1,0 2,0 3,0 2,2; do
      timeout -k 10 200 python bench.py $B --config $c --wave-prio $p > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $c $p"; tail -20 $O/ab.err; exit 1; }
      python -c "import json; d=json.load(open('$O/ab.json')); print('$rep $c $p', d['value'], {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','tree','verify','check','decode')})"
    done
  done
done
echo ok
