#!/bin/bash
# Round 4, the committed tree at the end of the round: GPU suite, smoke, the
# default bench and C4 once; then the commit / receive wave-priority pairs at
# C4 re-measured now that the receiver is the longer stream there (VERDICT r03
# item 4), interleaved, two repetitions.
set -o pipefail
O=gpurun_out/r04o; mkdir -p $O
line() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['decoded_ok'], d['values_ok'], (d.get('value_joined') or {}).get('value'), (d.get('valu_step') or {}).get('busy_4clk'), d['stage_ms'])" "$@"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|assert" $O/gputest.log | tail -30; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCHFAIL; tail -20 $O/bench_default.err; exit 1; }
line $O/bench_default.json default
Q="--no-cpu-baseline --no-pcie --no-joined-leg"
for rep in 1 2; do
  for wp in 0,2 0,3 1,2 0,1; do
    t=${wp/,/}
    timeout -k 10 300 python bench.py --config c4 --steps 60 --wave-prio $wp $Q > $O/c4_w${t}_$rep.json 2> $O/c4_w${t}_$rep.err || { echo BENCHFAIL $wp; tail -20 $O/c4_w${t}_$rep.err; exit 1; }
    line $O/c4_w${t}_$rep.json "c4 wave $wp"
  done
done
echo ok
