# Round 6: the decode join's stores.  A/B of the FFT decode's fused join:
# base (unaligned dword stores, default tile order), xcd (XCD-aware tile order
# for decode too), jal (aligned stores: v_alignbyte of neighbouring lanes),
# xjal (both).  Parity of the join first for each variant, then the bench's
# device legs at C4, C3, C1 and C2 (value = joined), twice each.
set -o pipefail
O=gpurun_out/${RUN:-r06r}; mkdir -p $O
R=$(pwd)
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
for lib in base xcd jal xjal; do
  if [ $lib = base ]; then unset RBC_GPU_LIB; else export RBC_GPU_LIB=$R/ab/librbc_gpu_$lib.so; fi
  timeout -k 10 300 $T tests/test_gpu_parity.py -k "fused_join or row_view or c4 or c1 or c3" > $O/tests_$lib.log 2>&1 || { echo TESTFAIL $lib; tail -30 $O/tests_$lib.log; exit 1; }
  tail -1 $O/tests_$lib.log
done
for rep in 1 2; do
  for cfg in c4 c3 c1 c2; do
    for lib in base xcd jal xjal; do
      if [ $lib = base ]; then unset RBC_GPU_LIB; else export RBC_GPU_LIB=$R/ab/librbc_gpu_$lib.so; fi
      timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-batcher --no-pcie --no-isolated > $O/${cfg}_${lib}_$rep.json 2> $O/${cfg}_${lib}_$rep.err || { echo BENCHFAIL $cfg $lib; tail -20 $O/${cfg}_${lib}_$rep.err; exit 1; }
      python -c "import json; d=json.load(open('$O/${cfg}_${lib}_$rep.json')); print('$cfg $lib $rep', d['value'], d['ms_per_step'], 'row', d['value_row_view']['value'], 'decode', d['stage_ms']['decode'], d['value_row_view']['stage_ms']['decode'], d['values_ok'], d['library'].split('/')[-1])"
    done
  done
done
echo ok
