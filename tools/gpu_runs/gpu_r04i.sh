#!/bin/bash
# Round 4: C4 LDS budget A/B.  merkle_path (receiver) and gf_regen (decode)
# share the CUs' LDS with the proposer's kernels under the two-stream
# pipeline: the product's 32 KiB branch stage (3 path blocks per CU, 150 KiB)
# leaves no room for a 31 KiB gf_regen block.  Variants (tools/build_ab.sh):
#   lvl28   : one sibling load per level, 28 KiB pad (3 blocks/CU, r04c's 355)
#   lvl20   : one sibling load per level, 20 KiB pad (4 blocks/CU)
#   lvl0    : one sibling load per level, no pad (8 blocks/CU)
#   jc8     : product path, gf_regen table chunks of 8 inputs (15 KiB)
#   lvl28jc8: lvl28 + jc8
# interleaved, two reps; then C2 base/jc8 (gf_regen's C2 form is W = 2).
set -o pipefail
O=gpurun_out/r04i; mkdir -p $O
R=$(pwd)
Q="--no-cpu-baseline --no-pcie --no-joined-leg"
run() {  # config variant rep
  if [ $2 = base ]; then L=""; else L=$R/ab/librbc_gpu_$2.so; fi
  RBC_GPU_LIB=$L timeout -k 10 300 python bench.py --config $1 --steps 60 $Q > $O/$1_$2_$3.json 2> $O/$1_$2_$3.err || { echo BENCHFAIL $1 $2; tail -20 $O/$1_$2_$3.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['decoded_ok'], d['values_ok'], d['oracle_sample_ok'], d['stage_ms'])" $O/$1_$2_$3.json "$1 $2"
}
for rep in 1 2; do
  for v in base lvl28 lvl20 lvl0 jc8 lvl28jc8; do run c4 $v $rep || exit 1; done
done
for rep in 1 2; do
  for v in base jc8; do run c2 $v $rep || exit 1; done
done
echo ok
