# Round 5: interpolate's joined value assembled by the FFT re-encode from the
# data rows it loads (no separate join pass): GPU suite, default bench twice
# (value_joined), and the joined form at C1 / C4.
set -o pipefail
O=gpurun_out/r05t; mkdir -p $O
Q="--no-cpu-baseline --no-pcie --no-batcher --no-joined-leg"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|assert" $O/gputest.log | tail -30; exit 1; }
tail -1 $O/gputest.log
for rep in 1 2; do
  timeout -k 10 600 python bench.py --no-batcher > $O/bench_default_$rep.json 2> $O/bench_default_$rep.err || { echo BENCHFAIL; tail -20 $O/bench_default_$rep.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); j=d['value_joined']; print('default', d['value'], 'joined', j['value'], j['values_ok'], j['stage_ms']['decode'], d['stage_ms']['decode'])" $O/bench_default_$rep.json
done
for cfg in c4 c1; do
  timeout -k 10 300 python bench.py --config $cfg --steps 60 --join $Q > $O/${cfg}_join.json 2> $O/${cfg}_join.err || { echo BENCHFAIL $cfg; tail -20 $O/${cfg}_join.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['values_ok'], d['decoded_ok'], d['config']['value_form'])" $O/${cfg}_join.json $cfg
done
echo ok
