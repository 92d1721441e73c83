#!/bin/bash
# Round 4: Merkle build tree packing A/B -- 4 trees per one-wave block at C4
# (8 at C2) instead of 2 (4): the narrow upper levels share a pass with more
# trees, at twice the node LDS.  Interleaved, C4 then C2.
set -o pipefail
O=gpurun_out/r04l; mkdir -p $O
R=$(pwd)
Q="--no-cpu-baseline --no-pcie --no-joined-leg"
run() {  # config variant rep
  if [ $2 = base ]; then L=""; else L=$R/ab/librbc_gpu_$2.so; fi
  RBC_GPU_LIB=$L timeout -k 10 300 python bench.py --config $1 --steps 60 $Q > $O/$1_$2_$3.json 2> $O/$1_$2_$3.err || { echo BENCHFAIL $1 $2; tail -20 $O/$1_$2_$3.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['decoded_ok'], d['values_ok'], d['oracle_sample_ok'], d['stage_ms'])" $O/$1_$2_$3.json "$1 $2"
}
for rep in 1 2; do
  for v in base g1024; do run c4 $v $rep || exit 1; done
done
for rep in 1 2; do
  for v in base g1024; do run c2 $v $rep || exit 1; done
done
echo ok
