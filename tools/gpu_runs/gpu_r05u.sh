# Round 5: cur's decode prepare on the aux stream beside prev's recheck (the
# decode's change flags double-buffered by parity): GPU suite, then A/B against
# the library before the change (ab/librbc_gpu_base.so) at C4, C2, C1, twice.
set -o pipefail
O=gpurun_out/r05u; mkdir -p $O
Q="--no-cpu-baseline --no-pcie --no-batcher --no-joined-leg"
line() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['decoded_ok'], d['values_ok'], d['oracle_sample_ok'], {k: d['stage_ms'][k] for k in ('verify','check','decode')})" "$@"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|assert" $O/gputest.log | tail -30; exit 1; }
tail -1 $O/gputest.log
for rep in 1 2; do
  for cfg in c4 c2 c1; do
    for v in new base; do
      L=""; [ $v = base ] && L=ab/librbc_gpu_base.so
      RBC_GPU_LIB=$L timeout -k 10 300 python bench.py --config $cfg --steps 60 $Q > $O/ab_${cfg}_${v}_$rep.json 2> $O/ab_${cfg}_${v}_$rep.err || { echo BENCHFAIL $cfg $v; tail -20 $O/ab_${cfg}_${v}_$rep.err; exit 1; }
      line $O/ab_${cfg}_${v}_$rep.json ab_${cfg}_${v}_$rep
    done
  done
done
echo ok
