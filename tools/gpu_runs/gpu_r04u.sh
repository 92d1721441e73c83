#!/bin/bash
# Round 4, final code (split W = 256 Merkle build): smoke, the default bench,
# C4, and C4's PMC (VALU, traffic) so the C4 line prices the final kernels.
set -o pipefail
O=gpurun_out/r04u; mkdir -p $O
line() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['decoded_ok'], d['values_ok'], (d.get('value_joined') or {}).get('value'), (d.get('valu_step') or {}).get('busy_4clk'), d['stage_ms'])" "$@"; }
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCHFAIL; tail -20 $O/bench_default.err; exit 1; }
line $O/bench_default.json default
Q="--no-cpu-baseline --no-pcie --no-joined-leg"
timeout -k 10 300 python bench.py --config c4 --steps 60 $Q > $O/c4.json 2> $O/c4.err || { echo BENCHFAIL c4; tail -20 $O/c4.err; exit 1; }
line $O/c4.json c4
PASSES="sq1 fetch write" bash tools/pmc_passes.sh r04u_c4 --config c4 --steps 5 --warmup 3 --no-isolated $Q || { echo PMCFAIL; exit 1; }
echo ok
