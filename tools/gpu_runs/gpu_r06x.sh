# Round 6: the coalescer's launches completed by their own thread (copies out
# of batch t beside the copies into batch t+1).  The batcher GPU tests, then
# the epoch by request kind, twice each (compare profiles/r06w/).
set -o pipefail
O=gpurun_out/${RUN:-r06x}; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_gpu_batcher.py tests/test_gpu_verified.py -k "batcher" > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for kinds in s i vi svi viK sviK; do
    timeout -k 10 300 tools/batcher_bench epoch 1024 16 8 200 - $kinds > $O/epoch_${kinds}_$rep.jsonl 2> $O/epoch_${kinds}_$rep.err || { echo EPOCHFAIL $kinds; tail -20 $O/epoch_${kinds}_$rep.err; exit 1; }
    python -c "import json; r=[json.loads(x) for x in open('$O/epoch_${kinds}_$rep.jsonl')]; print('$kinds', [(x['interpolate'].split()[0], x['GBps'], x['seconds'], x['launches']) for x in r if x['phase']=='epoch'])"
  done
done
echo ok
