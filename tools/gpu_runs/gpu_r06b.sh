# Round 6: the fused host receive (rbc_receive_batch), the C4 verify-on-proposer
# A/B, the batcher epoch's client window, and PMC of the
# interpolate row hashing with and without the validate leaves.
set -o pipefail
O=gpurun_out/r06b; mkdir -p $O
R=$(pwd)
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_verified.py tests/test_gpu_bench.py -k "verified or receive_batch or host_fed or noncodeword or batcher" > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
Q="--no-cpu-baseline --no-pcie --no-batcher --no-second-form --no-isolated"
for rep in 1 2; do
  for v in receiver proposer; do
    timeout -k 10 300 python bench.py --config c4 --verify-on $v $Q > $O/c4_$v$rep.json 2> $O/c4_$v$rep.err || { echo BENCHFAIL c4 $v; tail -20 $O/c4_$v$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/c4_$v$rep.json')); print('c4', '$v', d['value'], d['ms_per_step'], d['decoded_ok'], d['values_ok'], {k: round(x,3) for k,x in d['stage_ms'].items()})"
  done
done
for W in 8 32 64; do
  timeout -k 10 300 tools/batcher_bench epoch 1024 16 $W 200 > $O/epoch_w$W.jsonl 2> $O/epoch_w$W.err || { echo EPOCHFAIL $W; tail -20 $O/epoch_w$W.err; exit 1; }
  echo W=$W; cat $O/epoch_w$W.jsonl
done
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d $R/$O/pmc_interp -o run --output-format csv -- python3 $R/tools/pmc_interp_probe.py run 256 > $R/$O/pmc_interp.out 2> $R/$O/pmc_interp.err ) || { echo PMCFAIL; tail -20 $O/pmc_interp.err; exit 1; }
cat $O/pmc_interp.out
F=$(find $O/pmc_interp -name "*counter_collection.csv" | head -1)
python tools/pmc_interp_probe.py summary $F 256 > $O/pmc_interp_summary.json && cat $O/pmc_interp_summary.json
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCHFAIL; tail -30 $O/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_default.json')); p=d['pcie_inclusive']; print('value', d['value'], d['ms_per_step'], 'row', (d.get('value_row_view') or {}).get('value'), 'host', p['aggregate_GBps'], 'fused', p['fused']['aggregate_GBps'], p['rank0'].get('alone_GBps'), p['rank0']['pcie_GBps'], p['ok'], 'epoch', d['batcher']['epoch'])"
echo ok
