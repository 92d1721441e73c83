# Round 3, second session, first call: state of the committed code -- smoke,
# default bench, C4 / C1 benches, and C4 counter passes (pipelined and serial)
# for the GF-decode evidence VERDICT r02 item 3 asks for.
set -o pipefail
O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCHFAIL; tail -30 $O/bench_default.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench_default.json')); print(d['value'], d['ms_per_step'], d['vs_baseline'], d['stage_ms'], d['roofline']['frac'], d['roofline_decode']['frac'], d['roofline_encode']['frac'])"
B="--no-cpu-baseline --no-pcie --steps 40"
for c in c4 c1; do
  timeout -k 10 300 python bench.py $B --config $c > $O/$c.json 2>> $O/cfg.err || { echo CFGFAIL $c; tail -20 $O/cfg.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$c.json')); print('$c', d['value'], d['ms_per_step'], {k: round(v, 3) for k, v in d['stage_ms'].items()})"
done
P="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 4 --steps 10 --warmup 3"
timeout -k 10 500 bash tools/pmc_passes.sh r03g_c4 --config c4 $P > $O/c4p.log 2>&1 || { echo C4PFAIL; tail -20 $O/c4p.log; exit 1; }
timeout -k 10 500 bash tools/pmc_passes.sh r03g_c4s --config c4 --pipeline 0 $P > $O/c4s.log 2>&1 || { echo C4SFAIL; tail -20 $O/c4s.log; exit 1; }
echo ok
