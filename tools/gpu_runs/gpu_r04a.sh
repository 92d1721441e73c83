# Round 4, first GPU call: the poisoned-receive parity tests and bench guard
# (VERDICT r03 item 1), the mutant that must fail the guard, the dwordx4 / x3
# gf_regen stores (item 2): GPU suite, smoke(), the default bench.
set -o pipefail
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|error|assert" $O/gputest.log | tail -40; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCHFAIL; tail -30 $O/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_default.json')); print(d['value'], d['ms_per_step'], d['decoded_ok'], d['values_ok'], d['guard'], d['oracle_sample_ok'], d['roofline']['frac'], d['cpu_baseline']['value'])"
echo ok
