#!/bin/bash
# Round 4: C4 decode-transform issue levels re-measured after the path and
# recheck cuts (the receiver is now the longer stream at C4: verify + check +
# decode 8.55 ms against the proposer's 7.7).  --decode-prio GEMV,re-encode
# (c = commit level, r = receive level); the product's C4 default is r,c.
set -o pipefail
O=gpurun_out/r04m; mkdir -p $O
Q="--no-cpu-baseline --no-pcie --no-joined-leg"
for rep in 1 2; do
  for dp in r,c r,r c,r c,c; do
    t=${dp/,/}
    timeout -k 10 300 python bench.py --config c4 --steps 60 --decode-prio $dp $Q > $O/c4_${t}_$rep.json 2> $O/c4_${t}_$rep.err || { echo BENCHFAIL $dp; tail -20 $O/c4_${t}_$rep.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['decoded_ok'], d['values_ok'], d['stage_ms'])" $O/c4_${t}_$rep.json "c4 $dp"
  done
done
echo ok
