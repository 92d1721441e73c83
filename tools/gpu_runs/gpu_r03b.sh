# Round 3: GPU suite (new: C3 8192 single + 2-rank partition, C4 16384, row view,
# receive-step aliasing), smoke, default bench, and the row-view vs join A/B.
set -o pipefail
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu --maxfail=5 -v --timeout 600 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|error" $O/gputest.log | tail -30; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -30 $O/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCHFAIL; tail -30 $O/bench_default.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench_default.json')); print(d['value'], d['ms_per_step'], d['vs_baseline'], d['stage_ms'], d['roofline']['frac'], d['roofline_decode']['frac'], d['roofline_encode']['frac'])"
B="--no-cpu-baseline --no-pcie --steps 60"
for v in "--join" "" "--faults-on proposer" "--join" ""; do
  timeout -k 10 300 python bench.py $B $v > $O/ab.json 2>> $O/ab.err || { echo ABFAIL; tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('AB', '$v', d['value'], d['stage_ms'])"
done
echo ok
