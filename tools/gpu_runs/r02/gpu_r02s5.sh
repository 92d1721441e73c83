# Evidence at the current code: GPU suite, smoke, driver-style bench, rocprof trace + PMC (tag r02s5)
set -o pipefail
O=gpurun_out/r02s5; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
t0=$(date +%s.%N)
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCHFAIL; tail -30 $O/bench_default.err; exit 1; }
t1=$(date +%s.%N)
echo "bench wall seconds: $(python -c "print(round($t1-$t0,1))")"
python -c "
import json; d=json.load(open('$O/bench_default.json')); print(d['value'], d['ms_per_step'], d['vs_baseline'], d['values_ok'], d['oracle_sample_ok'], d['roofline']['frac'], d['commit_only']['GBps'], d['receive_only']['GBps'], d['cpu_baseline']['value'])"
timeout -k 10 900 bash tools/profile.sh r02s5 > $O/profile.log 2>&1 || { echo PROFFAIL; tail -30 $O/profile.log; exit 1; }
echo ok
