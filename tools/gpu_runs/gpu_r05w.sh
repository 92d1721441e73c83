# Round 5, final tree (fused join, lane sealing pause max_wait/4): the GPU suite, smoke() and the default bench twice on
# the final tree (the driver's own round-end steps), wall time of each.
set -o pipefail
O=gpurun_out/r05w; mkdir -p $O
TIMEFORMAT='%R s'
line() { python -c "import json,sys; d=json.load(open(sys.argv[1])); v=d.get('valu_step') or {}; b=d.get('batcher') or {}; print(sys.argv[2], d['value'], d['ms_per_step'], d['decoded_ok'], d['values_ok'], d['oracle_sample_ok'], (d.get('value_joined') or {}).get('value'), v.get('chain_frac_of_step'), [s['GBps'] for s in b.get('sweep', [])])" "$@"; }
{ time timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gputest.log 2>&1 ; } 2> $O/gputest.time || { echo TESTFAIL; grep -E "FAILED|Error|assert" $O/gputest.log | tail -30; exit 1; }
tail -1 $O/gputest.log; cat $O/gputest.time
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for rep in 1 2; do
  { time timeout -k 10 600 python bench.py > $O/bench_default_$rep.json 2> $O/bench_default_$rep.err ; } 2> $O/bench_default_$rep.time || { echo BENCHFAIL; tail -20 $O/bench_default_$rep.err; exit 1; }
  line $O/bench_default_$rep.json default; cat $O/bench_default_$rep.time
done
echo ok
