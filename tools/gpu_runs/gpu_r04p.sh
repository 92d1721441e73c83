#!/bin/bash
# Round 4: merkle_path with the speculative top levels and a two-level branch
# stage (16 KiB: 4 blocks per CU instead of 3) against the product's
# four-level stage; C4, interleaved, three repetitions.  The variant's own
# parity first: RBC_GPU_LIB points the verify tests at it.
set -o pipefail
O=gpurun_out/r04p; mkdir -p $O
R=$(pwd)
RBC_GPU_LIB=$R/ab/librbc_gpu_st2spec.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu -k "verify or recheck or receive_step" > $O/pytest.log 2>&1 || { echo PYTESTFAIL; grep -E "Error|assert|FAILED" $O/pytest.log | head -30; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
Q="--no-cpu-baseline --no-pcie --no-joined-leg"
run() {  # config variant rep
  if [ $2 = base ]; then L=""; else L=$R/ab/librbc_gpu_$2.so; fi
  RBC_GPU_LIB=$L timeout -k 10 300 python bench.py --config $1 --steps 60 $Q > $O/$1_$2_$3.json 2> $O/$1_$2_$3.err || { echo BENCHFAIL $1 $2; tail -20 $O/$1_$2_$3.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['decoded_ok'], d['values_ok'], d['oracle_sample_ok'], d['library'][-30:], d['stage_ms'])" $O/$1_$2_$3.json "$1 $2"
}
for rep in 1 2 3; do
  for v in base st2spec; do run c4 $v $rep || exit 1; done
done
echo ok
