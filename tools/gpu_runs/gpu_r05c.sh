# Round 5: the batcher's validate lane -- GPU test (16,384 outstanding vs the
# oracle) and the outstanding-validates sweep at C2.
set -o pipefail
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_batcher.py -x -v --timeout 200 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 400 tools/batcher_bench validate-sweep 256 16 200 1024 8192 32768 88064 > $O/sweep.jsonl 2> $O/sweep.err || { echo SWEEPFAIL; tail -20 $O/sweep.err; cat $O/sweep.jsonl; exit 1; }
cat $O/sweep.jsonl
timeout -k 10 300 tools/batcher_bench 1024 16 64 64 2048 200 > $O/all.jsonl 2> $O/all.err || { echo ALLFAIL; tail -20 $O/all.err; exit 1; }
cat $O/all.jsonl
echo ok
