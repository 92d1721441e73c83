# Round 5 A/B of the validate lane's sealing while launches run: quiet period
# max_wait/4 (va), and also the minimum arena age max_wait/2 (vb), against the
# product (max_wait for both), at 1k-88k outstanding, interleaved, twice.
set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
for rep in 1 2; do
  for v in prod va vb; do
    L=""; [ $v != prod ] && L=ab/$v
    LD_LIBRARY_PATH=$L${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 300 tools/batcher_bench validate-sweep 256 16 200 1024 8192 32768 88064 > $O/sweep_${v}_$rep.jsonl 2> $O/sweep_${v}_$rep.err || { echo SWEEPFAIL $v; tail -20 $O/sweep_${v}_$rep.err; exit 1; }
    python -c "import json,sys; r=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')]; print(sys.argv[2], [(x['outstanding'], x['GBps'], x['launches']) for x in r if x.get('phase')=='validate'], [x['failures'] for x in r if x.get('phase')=='check'])" $O/sweep_${v}_$rep.jsonl ${v}_$rep
  done
done
echo ok
