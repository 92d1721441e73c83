# Round 6: the value join as its own kernel on the aux stream (ab/nofj,
# RBC_FUSED_JOIN=0) against the FFT decode's fused join: C4, C1, C2 joined
# (device-resident), twice each; the join parity tests on the variant first.
set -o pipefail
O=gpurun_out/${RUN:-r06am}; mkdir -p $O
R=$(pwd)
RBC_GPU_LIB=$R/ab/nofj/librbc_gpu.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "fused_join or row_view or c4" > $O/tests_nofj.txt 2>&1 || { echo TESTFAIL; tail -30 $O/tests_nofj.txt; exit 1; }
tail -1 $O/tests_nofj.txt
Q="--no-cpu-baseline --no-batcher --no-pcie --no-isolated"
for rep in 1 2; do
  for cfg in c4 c1 c2; do
    for lib in base nofj; do
      if [ $lib = base ]; then unset RBC_GPU_LIB; else export RBC_GPU_LIB=$R/ab/nofj/librbc_gpu.so; fi
      timeout -k 10 300 python bench.py --config $cfg $Q > $O/${cfg}_${lib}_$rep.json 2> $O/${cfg}_${lib}_$rep.err || { echo BENCHFAIL; tail -20 $O/${cfg}_${lib}_$rep.err; exit 1; }
      python -c "import json; d=json.load(open('$O/${cfg}_${lib}_$rep.json')); print('$cfg $lib $rep', d['value'], d['ms_per_step'], 'row', d['value_row_view']['value'], 'decode', d['stage_ms']['decode'], 'interp', d['stage_ms']['interp'], d['values_ok'])"
    done
  done
done
echo ok
