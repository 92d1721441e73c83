# Round 5: the proposer refills batch t-2's shard set once its recheck is done
# (rbc_rx_marks.prev_released, ABI 5) instead of after the whole receive step:
# GPU suite (incl. the clobber-after-release parity test), then A/B
# recheck / step at C4, C2, C1, interleaved, twice.
set -o pipefail
O=gpurun_out/r05q; mkdir -p $O
Q="--no-cpu-baseline --no-pcie --no-batcher --no-joined-leg"
line() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['decoded_ok'], d['values_ok'], d['oracle_sample_ok'], d['config'].get('set_release'))" "$@"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|assert" $O/gputest.log | tail -30; exit 1; }
tail -1 $O/gputest.log
for rep in 1 2; do
  for cfg in c4 c2 c1; do
    for rl in recheck step; do
      timeout -k 10 300 python bench.py --config $cfg --steps 60 --p-release $rl $Q > $O/ab_${cfg}_${rl}_$rep.json 2> $O/ab_${cfg}_${rl}_$rep.err || { echo BENCHFAIL $cfg $rl; tail -20 $O/ab_${cfg}_${rl}_$rep.err; exit 1; }
      line $O/ab_${cfg}_${rl}_$rep.json ab_${cfg}_${rl}_$rep
    done
  done
done
echo ok
