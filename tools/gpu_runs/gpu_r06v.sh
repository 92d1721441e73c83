# Round 6, ABI 7: the batcher epoch's kept pass against the verified pass,
# three processes each way (the epoch spreads 9-16 GB/s run to run), and the
# kept passes alone in a process (sviK).
set -o pipefail
O=gpurun_out/${RUN:-r06v}; mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 300 tools/batcher_bench epoch 1024 16 8 200 > $O/epoch_$rep.jsonl 2> $O/epoch_$rep.err || { echo EPOCHFAIL; tail -20 $O/epoch_$rep.err; exit 1; }
  python -c "import json; r=[json.loads(x) for x in open('$O/epoch_$rep.jsonl')]; print('all', [(x['interpolate'].split()[0], x['GBps']) for x in r if x['phase']=='epoch'])"
  timeout -k 10 300 tools/batcher_bench epoch 1024 16 8 200 - sviK > $O/epochK_$rep.jsonl 2> $O/epochK_$rep.err || { echo EPOCHFAIL; tail -20 $O/epochK_$rep.err; exit 1; }
  python -c "import json; r=[json.loads(x) for x in open('$O/epochK_$rep.jsonl')]; print('K', [(x['interpolate'].split()[0], x['GBps']) for x in r if x['phase']=='epoch'])"
done
echo ok
