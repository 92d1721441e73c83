#!/bin/bash
# Round 4: the W = 256 Merkle build split in two -- merkle_kernel<false> down
# to the layer of 32 nodes, merkle_top_kernel for the top five layers of 8
# trees per wave (roots + branch levels 4..7).  Full GPU suite first, then C4
# A/B against the one-kernel build (ab/librbc_gpu_notop.so), interleaved, and
# the product's VALU at C4.
set -o pipefail
O=gpurun_out/r04t; mkdir -p $O
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|assert" $O/gputest.log | tail -30; exit 1; }
tail -1 $O/gputest.log
Q="--no-cpu-baseline --no-pcie --no-joined-leg"
run() {  # config variant rep
  if [ $2 = base ]; then L=""; else L=$R/ab/librbc_gpu_$2.so; fi
  RBC_GPU_LIB=$L timeout -k 10 300 python bench.py --config $1 --steps 60 $Q > $O/$1_$2_$3.json 2> $O/$1_$2_$3.err || { echo BENCHFAIL $1 $2; tail -20 $O/$1_$2_$3.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['decoded_ok'], d['values_ok'], d['oracle_sample_ok'], d['stage_ms'])" $O/$1_$2_$3.json "$1 $2"
}
for rep in 1 2 3; do
  for v in base notop; do run c4 $v $rep || exit 1; done
done
for v in base notop; do run c2 $v 1 || exit 1; done
PASSES="sq1" bash tools/pmc_passes.sh r04t_c4 --config c4 --steps 5 --warmup 3 --no-isolated $Q || { echo PMCFAIL; exit 1; }
echo ok
