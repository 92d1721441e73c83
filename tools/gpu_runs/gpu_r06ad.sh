# Round 6: host batch API after the value repack and the short-row gathers:
# the verified / kept / pinned-pitch GPU tests, then C4 and C2 host-fed epochs
# twice each (compare profiles/r06ac/).
set -o pipefail
O=gpurun_out/${RUN:-r06ad}; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_gpu_verified.py tests/test_gpu_parity.py -k "verified or kept or keep or pitch or receive or interpolate" > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for cfg in c4 c2 c1; do
    ni=$([ $cfg = c4 ] && echo 16384 || echo 1024)
    timeout -k 10 300 python tools/host_bench.py --config $cfg --epoch $ni > $O/host_${cfg}_$rep.json 2> $O/host_${cfg}_$rep.err || { echo HOSTFAIL; tail -20 $O/host_${cfg}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/host_${cfg}_$rep.json')); print('$cfg $rep', 'drop-in', d['GBps'], 'kept', d['kept']['GBps'], 'fused', d['fused']['GBps'], d['ok'], d['alone_GBps'])"
  done
done
echo ok
