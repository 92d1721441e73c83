# Round 5: receive step without memset / D2D launches on the receiver stream
# (ping-pong list counters zeroed by the hashing launch, roots kept by the
# compaction) -- GPU suite, smoke, default bench, C4; then the validate-lane
# parameter sweep (gpu_r05e.sh).
set -o pipefail
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|error|assert" $O/gputest.log | tail -40; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
line() { python -c "import json,sys; d=json.load(open(sys.argv[1])); v=d.get('valu_step') or {}; print(sys.argv[2], d['value'], d['ms_per_step'], d['decoded_ok'], d['values_ok'], v.get('chain_frac_of_step'), v.get('issue_frac_of_step'), {k: round(x,3) for k,x in d['stage_ms'].items()})" "$@"; }
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCHFAIL; tail -20 $O/bench_default.err; exit 1; }
line $O/bench_default.json default
python -c "import json; d=json.load(open('$O/bench_default.json')); print(json.dumps(d.get('batcher'))[:1500])"
timeout -k 10 300 python bench.py --config c4 --steps 60 --no-joined-leg --no-cpu-baseline --no-pcie > $O/c4.json 2> $O/c4.err || { echo BENCHFAIL c4; tail -20 $O/c4.err; exit 1; }
line $O/c4.json c4
bash tools/gpu_runs/gpu_r05e.sh
