# Round 3, final tree (gf_regen with exact row counts): GPU suite,
# smoke, the default bench (twice), C1 / C3 / C4 lines, rocprof evidence (C2
# trace + PMC via tools/profile.sh; C4 pipelined and C2 / C4 serial trace + PMC
# via tools/pmc_passes.sh: each kernel alone).
set -o pipefail
O=gpurun_out/r03zk; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|error" $O/gputest.log | tail -30; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for rep in 1 2; do
  timeout -k 10 400 python bench.py > $O/bench_default_$rep.json 2> $O/bench_default.err || { echo BENCHFAIL; tail -30 $O/bench_default.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/bench_default_$rep.json')); print(d['value'], d['ms_per_step'], d['vs_baseline'], d['stage_ms'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['traffic'], d['roofline_decode']['frac'], d['roofline_decode']['traffic'], d['roofline_encode']['frac'])"
done
B="--no-cpu-baseline --no-pcie --steps 60"
for c in c1 c3 c4; do
  timeout -k 10 300 python bench.py $B --config $c > $O/$c.json 2>> $O/cfg.err || { echo CFGFAIL $c; tail -20 $O/cfg.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$c.json')); print('$c', d['value'], d['ms_per_step'], {k: round(v, 3) for k, v in d['stage_ms'].items()})"
done
timeout -k 10 900 bash tools/profile.sh r03zk --steps 20 --warmup 3 > $O/prof.log 2>&1 || { echo PROFFAIL; tail -20 $O/prof.log; exit 1; }
P="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 4 --steps 10 --warmup 3"
timeout -k 10 500 bash tools/pmc_passes.sh r03zk_c4 --config c4 $P > $O/c4p.log 2>&1 || { echo C4PFAIL; tail -20 $O/c4p.log; exit 1; }
S="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2 --steps 5 --warmup 2 --pipeline 0"
timeout -k 10 500 bash tools/pmc_passes.sh r03zk_c4s --config c4 $S > $O/c4s.log 2>&1 || { echo C4SFAIL; tail -20 $O/c4s.log; exit 1; }
timeout -k 10 500 bash tools/pmc_passes.sh r03zk_c2s --config c2 $S > $O/c2s.log 2>&1 || { echo C2SFAIL; tail -20 $O/c2s.log; exit 1; }
echo ok
