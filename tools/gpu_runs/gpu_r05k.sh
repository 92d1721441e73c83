# Round 5 evidence: GPU suite, smoke, the default bench twice (with the
# batcher key), C1 / C3 / C4 lines, C3 at 8,192 on one GPU, and the rocprof
# kernel trace + stats of exactly `python bench.py`; A/B of the forked
# regen hashing (rbc_ctx_set_regen_hashing) at C4, C2, C1.
set -o pipefail
O=gpurun_out/r05k; mkdir -p $O
R=$(pwd)
Q="--no-cpu-baseline --no-pcie --no-batcher"
line() { python -c "import json,sys; d=json.load(open(sys.argv[1])); v=d.get('valu_step') or {}; print(sys.argv[2], d['value'], d['ms_per_step'], d['decoded_ok'], d['values_ok'], (d.get('value_joined') or {}).get('value'), v.get('chain_frac_of_step'), v.get('issue_frac_of_step'))" "$@"; }
timeout -k 10 60 tools/gf_probe 2.4 > $O/gf_probe.txt 2>&1 || { echo GFPROBEFAIL; cat $O/gf_probe.txt; exit 1; }
cat $O/gf_probe.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|error|assert" $O/gputest.log | tail -40; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for rep in 1 2; do
  timeout -k 10 500 python bench.py > $O/bench_default_$rep.json 2> $O/bench_default_$rep.err || { echo BENCHFAIL; tail -20 $O/bench_default_$rep.err; exit 1; }
  line $O/bench_default_$rep.json default
done
for cfg in c1 c3 c4; do
  timeout -k 10 300 python bench.py --config $cfg --steps 60 --no-joined-leg $Q > $O/$cfg.json 2> $O/$cfg.err || { echo BENCHFAIL $cfg; tail -20 $O/$cfg.err; exit 1; }
  line $O/$cfg.json $cfg
done
# A/B: the regenerated rows hashed on the aux stream (RBC_REGEN_FORK) against inline
for rep in 1 2; do
  for cfg in c4 c2 c1; do
    for rg in inline fork; do
      timeout -k 10 300 python bench.py --config $cfg --steps 60 --no-joined-leg --regen $rg $Q > $O/ab_${cfg}_${rg}_$rep.json 2> $O/ab_${cfg}_${rg}_$rep.err || { echo BENCHFAIL ab $cfg $rg; tail -20 $O/ab_${cfg}_${rg}_$rep.err; exit 1; }
      line $O/ab_${cfg}_${rg}_$rep.json ab_${cfg}_${rg}_$rep
    done
  done
done
timeout -k 10 600 python bench.py --config c3 --total-instances 8192 --steps 4 --warmup 1 --no-joined-leg $Q > $O/c3_8192.json 2> $O/c3_8192.err || { echo BENCHFAIL c3_8192; tail -20 $O/c3_8192.err; exit 1; }
line $O/c3_8192.json c3_8192
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof_default -o run --output-format csv -- python3 $R/bench.py > $R/$O/prof_default.json 2> $R/$O/prof_default.err ) || { echo PROFFAIL; tail -20 $O/prof_default.err; exit 1; }
line $O/prof_default.json profiled_default
echo ok
