#!/bin/bash
# Round 4: two proposer streams (consecutive batches' commits overlap, four
# shard sets) against one, C1 (one SHA wave per SIMD per stream: dependency-
# bound) and C2 / C4; interleaved, two repetitions.
set -o pipefail
O=gpurun_out/r04r; mkdir -p $O
Q="--no-cpu-baseline --no-pcie --no-joined-leg"
for rep in 1 2; do
  for cfg in c1 c2 c4; do
    for np in 1 2; do
      timeout -k 10 300 python bench.py --config $cfg --steps 60 --proposers $np $Q > $O/${cfg}_p${np}_$rep.json 2> $O/${cfg}_p${np}_$rep.err || { echo BENCHFAIL $cfg $np; tail -20 $O/${cfg}_p${np}_$rep.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['decoded_ok'], d['values_ok'], d['oracle_sample_ok'], d['stage_ms'])" $O/${cfg}_p${np}_$rep.json "$cfg p$np"
    done
  done
done
echo ok
