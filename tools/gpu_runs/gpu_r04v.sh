#!/bin/bash
# Round 4: C1's leaf hashing two rows per lane (sha_rows2_kernel, the two
# compressions interleaved) against one: at N = 64 the launch holds one wave
# per SIMD, where ILP may stand in for waves.  Interleaved, three repetitions.
set -o pipefail
O=gpurun_out/r04v; mkdir -p $O
R=$(pwd)
Q="--no-cpu-baseline --no-pcie --no-joined-leg"
run() {  # config variant rep
  if [ $2 = base ]; then L=""; else L=$R/ab/librbc_gpu_$2.so; fi
  RBC_GPU_LIB=$L timeout -k 10 300 python bench.py --config $1 --steps 60 $Q > $O/$1_$2_$3.json 2> $O/$1_$2_$3.err || { echo BENCHFAIL $1 $2; tail -20 $O/$1_$2_$3.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['decoded_ok'], d['values_ok'], d['oracle_sample_ok'], d['stage_ms'])" $O/$1_$2_$3.json "$1 $2"
}
for rep in 1 2 3; do
  for v in base rows2; do run c1 $v $rep || exit 1; done
done
echo ok
