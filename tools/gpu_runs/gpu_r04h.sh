# Round 4, final code: GPU suite, smoke, the default bench twice, the other
# configs, C3 at 8,192 on one GPU; rocprofv3 kernel trace + stats of exactly
# the driver's default command; PMC (VALU, traffic) at C2 and C4 and each
# kernel's loaded clock (serial schedule) -- the evidence in profiles/r04h_*.
set -o pipefail
O=gpurun_out/r04h; mkdir -p $O
R=$(pwd)
Q="--no-cpu-baseline --no-pcie"
line() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['decoded_ok'], d['values_ok'], (d.get('value_joined') or {}).get('value'), (d.get('valu_step') or {}).get('busy_4clk'), d['stage_ms'])" "$@"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|error|assert" $O/gputest.log | tail -40; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for rep in 1 2; do
  timeout -k 10 400 python bench.py > $O/bench_default_$rep.json 2> $O/bench_default_$rep.err || { echo BENCHFAIL; tail -20 $O/bench_default_$rep.err; exit 1; }
  line $O/bench_default_$rep.json default
done
for cfg in c1 c3 c4; do
  timeout -k 10 300 python bench.py --config $cfg --steps 60 --no-joined-leg $Q > $O/$cfg.json 2> $O/$cfg.err || { echo BENCHFAIL $cfg; tail -20 $O/$cfg.err; exit 1; }
  line $O/$cfg.json $cfg
done
timeout -k 10 600 python bench.py --config c3 --total-instances 8192 --steps 4 --warmup 1 --no-joined-leg $Q > $O/c3_8192.json 2> $O/c3_8192.err || { echo BENCHFAIL c3_8192; tail -20 $O/c3_8192.err; exit 1; }
line $O/c3_8192.json c3_8192
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof_default -o run --output-format csv -- python3 $R/bench.py > $R/$O/prof_default.json 2> $R/$O/prof_default.err ) || { echo PROFFAIL; tail -20 $O/prof_default.err; exit 1; }
line $O/prof_default.json profiled_default
PASSES="sq1 fetch write" bash tools/pmc_passes.sh r04h_c2 --steps 5 --warmup 3 --no-isolated --no-joined-leg $Q || { echo PMCFAIL c2; exit 1; }
PASSES="sq1 fetch write" bash tools/pmc_passes.sh r04h_c4 --config c4 --steps 5 --warmup 3 --no-isolated --no-joined-leg $Q || { echo PMCFAIL c4; exit 1; }
PASSES="sq1 sq2" bash tools/pmc_passes.sh r04h_c2s --pipeline 0 --steps 5 --warmup 3 --no-isolated --no-joined-leg $Q || { echo PMCFAIL c2s; exit 1; }
PASSES="sq1 sq2" bash tools/pmc_passes.sh r04h_c4s --config c4 --pipeline 0 --steps 5 --warmup 3 --no-isolated --no-joined-leg $Q || { echo PMCFAIL c4s; exit 1; }
echo ok
