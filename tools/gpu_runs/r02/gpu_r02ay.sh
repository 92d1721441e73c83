set -o pipefail
mkdir -p gpurun_out/r02ay
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02ay/gputest.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r02ay/gputest.log; exit 1; }
tail -1 gpurun_out/r02ay/gputest.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > gpurun_out/r02ay/smoke.log 2>&1 || { echo SMOKEFAIL; tail -30 gpurun_out/r02ay/smoke.log; exit 1; }
tail -1 gpurun_out/r02ay/smoke.log
t0=$(date +%s.%N)
timeout -k 10 400 python bench.py > gpurun_out/r02ay/bench_default.json 2> gpurun_out/r02ay/bench_default.err || { echo BENCHFAIL; tail -30 gpurun_out/r02ay/bench_default.err; exit 1; }
t1=$(date +%s.%N)
echo "bench wall seconds: $(python -c "print(round($t1-$t0,1))")"
python -c "
import json; d=json.load(open('gpurun_out/r02ay/bench_default.json')); print(d['value'], d['ms_per_step'], d['vs_baseline'], d['values_ok'], d['oracle_sample_ok'], d['roofline']['frac'], d['roofline']['isolated']['valu_frac_of_attainable'], d['commit_only']['GBps'], d['receive_only']['GBps'], d['pcie_inclusive']['shard_commit_GBps'], d['pcie_inclusive']['interpolate_GBps'])"
