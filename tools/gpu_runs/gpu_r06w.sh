# Round 6: what binds the batcher epoch?  The epoch with one or two request
# kinds at a time (s = shard, v = validate, i = interpolate; K = the kept
# passes alone), twice each.
set -o pipefail
O=gpurun_out/${RUN:-r06w}; mkdir -p $O
for rep in 1 2; do
  for kinds in s v i vi sv svi viK sviK; do
    timeout -k 10 300 tools/batcher_bench epoch 1024 16 8 200 - $kinds > $O/epoch_${kinds}_$rep.jsonl 2> $O/epoch_${kinds}_$rep.err || { echo EPOCHFAIL $kinds; tail -20 $O/epoch_${kinds}_$rep.err; exit 1; }
    python -c "import json; r=[json.loads(x) for x in open('$O/epoch_${kinds}_$rep.jsonl')]; print('$kinds', [(x['interpolate'].split()[0], x['GBps'], x['seconds'], x['launches']) for x in r if x['phase']=='epoch'])"
  done
done
echo ok
