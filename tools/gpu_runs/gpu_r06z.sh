# Round 6: the batcher epoch against the client window (instances each of the
# 16 client threads keeps in flight), full mix, twice each.
set -o pipefail
O=gpurun_out/${RUN:-r06z}; mkdir -p $O
for rep in 1 2; do
  for w in ${WS:-4 8 16 32}; do
    timeout -k 10 300 tools/batcher_bench epoch 1024 16 $w 200 > $O/epoch_w${w}_$rep.jsonl 2> $O/epoch_w${w}_$rep.err || { echo EPOCHFAIL $w; tail -20 $O/epoch_w${w}_$rep.err; exit 1; }
    python -c "import json; r=[json.loads(x) for x in open('$O/epoch_w${w}_$rep.jsonl')]; print('w$w', [(x['interpolate'].split()[0], x['GBps'], x['launches']) for x in r if x['phase']=='epoch'])"
  done
done
echo ok
