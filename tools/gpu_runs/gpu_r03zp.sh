# Round 3: the N = 128 FFT kernels held to 128 VGPRs (4 waves per SIMD:
# waves_per_eu(4), decode compare group GD = 1; encode 125 -> 128, decode
# 152 -> 128, no scratch; ab/librbc_gpu_fft4.so) against the product, C2 / C3,
# with the GPU parity tests on the candidate first; order alternated.
set -o pipefail
O=gpurun_out/r03zp; mkdir -p $O
R=$GRAFT_REPO_ROOT
RBC_GPU_LIB_AB=$R/ab/librbc_gpu_fft4.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py > $O/parity.log 2>&1 || { echo PARITYFAIL; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2"
for rep in 1 2 3 4; do
  order="fft4 new"; [ $((rep % 2)) = 0 ] && order="new fft4"
  for cv in "c2 --steps 100" "c3 --steps 30"; do
    c=${cv%% *}; extra=${cv#* }
    for v in $order; do
      lib=""; [ $v != new ] && lib=$R/ab/librbc_gpu_$v.so
      RBC_GPU_LIB_AB=$lib timeout -k 10 200 python bench.py $B --config $c $extra > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $c $v"; tail -20 $O/ab.err; exit 1; }
      python -c "import json; d=json.load(open('$O/ab.json')); print('$rep $c $v', d['value'], d['values_ok'], {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','tree','verify','check','decode')})"
    done
  done
done
echo ok
