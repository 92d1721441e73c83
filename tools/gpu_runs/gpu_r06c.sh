# Round 6: do H2D and D2H overlap on this box's PCIe link (SDMA vs kernel-driven copies)?
set -o pipefail
O=gpurun_out/r06c; mkdir -p $O
for b in 64 256 1024; do
  timeout -k 10 120 tools/probes/duplex_probe 1024 $b > $O/duplex_b$b.json 2> $O/duplex_b$b.err || { echo PROBEFAIL; cat $O/duplex_b$b.err; exit 1; }
  cat $O/duplex_b$b.json
done
echo ok
