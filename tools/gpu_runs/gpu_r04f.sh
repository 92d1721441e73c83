# Round 4: merkle_path_kernel with its four branch levels staged in LDS (3
# blocks per CU): GPU suite, smoke, default bench; C4 (x3), C1, C3 lines;
# PMC (VALU, traffic) at C4 and each kernel's loaded clock at C4 (serial).
set -o pipefail
O=gpurun_out/r04f; mkdir -p $O
Q="--no-cpu-baseline --no-pcie"
line() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['decoded_ok'], d['values_ok'], (d.get('value_joined') or {}).get('value'), (d.get('valu_step') or {}).get('busy_4clk'), d['stage_ms'])" "$@"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|error|assert" $O/gputest.log | tail -40; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCHFAIL; tail -20 $O/bench_default.err; exit 1; }
line $O/bench_default.json default
for run in c4_1 c1 c4_2 c3 c4_3; do
  cfg=${run%_*}
  timeout -k 10 300 python bench.py --config $cfg --steps 60 --no-joined-leg $Q > $O/$run.json 2> $O/$run.err || { echo BENCHFAIL $run; tail -20 $O/$run.err; exit 1; }
  line $O/$run.json $run
done
PASSES="sq1 fetch write" bash tools/pmc_passes.sh r04f_c4 --config c4 --steps 5 --warmup 3 --no-isolated --no-joined-leg $Q || { echo PMCFAIL c4; exit 1; }
PASSES="sq1 sq2" bash tools/pmc_passes.sh r04f_c4s --config c4 --pipeline 0 --steps 5 --warmup 3 --no-isolated --no-joined-leg $Q || { echo PMCFAIL c4s; exit 1; }
bash tools/gpu_runs/gpu_r04g.sh || { echo R04GFAIL; exit 1; }
echo ok
