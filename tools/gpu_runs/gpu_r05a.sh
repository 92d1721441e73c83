# Round 5, first run: the GPU suite (the recheck fix for Byzantine padding
# nodes, rx marks ABI 4, the 8-rank rehearsal), smoke, the default bench.
set -o pipefail
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|error|assert" $O/gputest.log | tail -40; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCHFAIL; tail -20 $O/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_default.json')); print(d['value'], d['ms_per_step'], d['decoded_ok'], d['values_ok'], d['stage_ms'])"
echo ok
