# Round 3: the bench line after vs_baseline -> null (cpu_baseline.gpu_over_cpu):
# bench GPU tests, smoke, one default run.
set -o pipefail
O=gpurun_out/r03zc; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bench.py > $O/t.log 2>&1 || { echo TFAIL; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCHFAIL; tail -30 $O/bench_default.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench_default.json')); print(d['value'], d['vs_baseline'], d['vs_baseline_basis'], d['cpu_baseline']['value'], d['cpu_baseline']['gpu_over_cpu'], d['config']['wave_priority'])"
echo ok
