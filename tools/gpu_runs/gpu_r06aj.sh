# Round 6: is the batcher epoch's leaves-reused pass slower than the full
# rehash, or only the first timed pass?  verified, full, then full, verified
# again in the same process (RBC_EPOCH_ORDER_CHECK), three processes.
set -o pipefail
O=gpurun_out/${RUN:-r06aj}; mkdir -p $O
for rep in 1 2 3; do
  RBC_EPOCH_ORDER_CHECK=1 timeout -k 10 300 tools/batcher_bench epoch 1024 16 64 200 - svi 0 > $O/epoch_$rep.jsonl 2> $O/epoch_$rep.err || { echo EPOCHFAIL; tail -20 $O/epoch_$rep.err; exit 1; }
  python -c "import json; r=[json.loads(x) for x in open('$O/epoch_$rep.jsonl')]; print([(x['interpolate'], x['GBps']) for x in r if x['phase']=='epoch'])"
done
echo ok
