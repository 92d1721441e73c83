# Round 6: do H2D and D2H overlap on this box's PCIe link (SDMA vs kernel-driven
# copies)?  And the host API's slot count (4 vs 8, ab/s8) under the host-fed
# epoch and the batcher's drop-in epoch, with the epoch's per-kind breakdown.
set -o pipefail
O=gpurun_out/r06c; mkdir -p $O
for b in 64 256 1024; do
  timeout -k 10 120 tools/probes/duplex_probe 1024 $b > $O/duplex_b$b.json 2> $O/duplex_b$b.err || { echo PROBEFAIL; cat $O/duplex_b$b.err; exit 1; }
  cat $O/duplex_b$b.json
done
for lib in base s8; do
  if [ $lib = s8 ]; then export RBC_GPU_LIB=$(pwd)/ab/s8/librbc_gpu.so LD_LIBRARY_PATH=$(pwd)/ab/s8; fi
  for infl in 2 3; do
    timeout -k 10 300 python tools/host_bench.py --epoch 1024 --inflight $infl > $O/host_${lib}_i$infl.json 2> $O/host_${lib}_i$infl.err || { echo HOSTFAIL; tail -20 $O/host_${lib}_i$infl.err; exit 1; }
    python -c "import json; d=json.load(open('$O/host_${lib}_i$infl.json')); print('$lib', 'inflight $infl', d['library'][-30:], d['GBps'], d['fused']['GBps'], d['alone_GBps'], d['pcie_GBps'], d['fused']['pcie_GBps'], d['ok'])"
  done
  for kinds in svi s v vi; do
    timeout -k 10 300 tools/batcher_bench epoch 1024 16 8 200 - $kinds > $O/epoch_${lib}_$kinds.jsonl 2> $O/epoch_${lib}_$kinds.err || { echo EPOCHFAIL; tail -20 $O/epoch_${lib}_$kinds.err; exit 1; }
    echo $lib $kinds; grep -v '"phase": "check"' $O/epoch_${lib}_$kinds.jsonl | python -c "import sys, json; [print(' ', (d:=json.loads(l))['interpolate'], d['seconds'], d['GBps'], d['launches']) for l in sys.stdin]"
  done
done
echo ok
