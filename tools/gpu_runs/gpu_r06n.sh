# Round 6: the host-fed epoch with the proposer and the receiver side on one
# context (4 host slots, one lock) against a context each.
set -o pipefail
O=gpurun_out/r06n; mkdir -p $O
for rep in 1 2; do
  for cfg in c2 c4; do
    inst=1024; [ $cfg = c4 ] && inst=16384
    for cx in 1 2; do
      timeout -k 10 300 python tools/host_bench.py --config $cfg --epoch $inst --inflight 2 --contexts $cx > $O/host_${cfg}_x${cx}_$rep.json 2> $O/host_${cfg}_x${cx}_$rep.err || { echo HOSTFAIL; tail -20 $O/host_${cfg}_x${cx}_$rep.err; exit 1; }
      python -c "import json; d=json.load(open('$O/host_${cfg}_x${cx}_$rep.json')); print('$cfg', 'contexts $cx', d['GBps'], d['fused']['GBps'], d['pcie_GBps'], d['fused']['pcie_GBps'], d['ok'])"
    done
  done
done
echo ok
