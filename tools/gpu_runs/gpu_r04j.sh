#!/bin/bash
# Round 4: merkle_path's branch stage with its loads batched (8 or 16 per
# lane in flight, raw buffer loads, no per-piece branch): the r04f stage
# waited on every 16-B load.  GPU parity first, then C4 A/B, interleaved:
#   base    : 4 levels staged (32 KiB, 3 blocks/CU), 8 loads in flight
#   st4sb16 : 16 in flight
#   st2     : 2 levels staged (16 KiB, 4 blocks/CU)
#   st2sb16 : st2, 16 in flight
#   lvl20   : r04i's best: one sibling load per level, 20 KiB pad
#   st2jc8  : st2 + gf_regen table chunks of 8 inputs
set -o pipefail
O=gpurun_out/r04j; mkdir -p $O
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTESTFAIL; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
Q="--no-cpu-baseline --no-pcie --no-joined-leg"
run() {  # config variant rep
  if [ $2 = base ]; then L=""; else L=$R/ab/librbc_gpu_$2.so; fi
  RBC_GPU_LIB=$L timeout -k 10 300 python bench.py --config $1 --steps 60 $Q > $O/$1_$2_$3.json 2> $O/$1_$2_$3.err || { echo BENCHFAIL $1 $2; tail -20 $O/$1_$2_$3.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['decoded_ok'], d['values_ok'], d['oracle_sample_ok'], d['stage_ms'])" $O/$1_$2_$3.json "$1 $2"
}
for rep in 1 2; do
  for v in base st4sb16 st2 st2sb16 lvl20 st2jc8; do run c4 $v $rep || exit 1; done
done
echo ok
