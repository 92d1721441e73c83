# Round 3: N = 256 FFT without the top-layer copy of the coefficient rows
# (product: 190 / 179 VGPRs, 2 waves per SIMD) and the same capped at 3 waves
# per SIMD (ab/librbc_gpu_fftwpe3.so: 168 VGPRs, 16 / 39 spilled dwords)
# against the committed kernels (ab/librbc_gpu_head.so: 250 / 256 VGPRs):
# parity of both new builds, each kernel alone (serial trace), pipelined benches.
set -o pipefail
O=gpurun_out/r03zb; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py > $O/parity.log 2>&1 || { echo PARITYFAIL; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
RBC_GPU_LIB_AB=$R/ab/librbc_gpu_fftwpe3.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py > $O/parity3.log 2>&1 || { echo PARITY3FAIL; tail -30 $O/parity3.log; exit 1; }
tail -1 $O/parity3.log
cd /tmp && export TMPDIR=/tmp
Q="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2 --pipeline 0 --steps 5 --warmup 2"
for v in new fftwpe3 head; do
  lib=""; [ $v != new ] && lib=$R/ab/librbc_gpu_$v.so
  for c in c4 c2; do
    RBC_GPU_LIB_AB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/t_${c}_$v -o run --output-format csv -- python3 $R/bench.py --config $c $Q > /dev/null 2> $R/$O/t.log || { echo "TFAIL $v $c"; tail -5 $R/$O/t.log; exit 1; }
    grep -h "rs_fft" $R/$O/t_${c}_$v/run_kernel_stats.csv | cut -d, -f1-4 | sed "s/^/$c $v /"
  done
done
cd $R
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2"
for rep in 1 2; do
  for cv in "c4 --steps 40" "c2 --steps 100" "c1 --steps 60"; do
    c=${cv%% *}; extra=${cv#* }
    for v in new fftwpe3 head; do
      lib=""; [ $v != new ] && lib=$R/ab/librbc_gpu_$v.so
      RBC_GPU_LIB_AB=$lib timeout -k 10 200 python bench.py $B --config $c $extra > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $c $v"; tail -20 $O/ab.err; exit 1; }
      python -c "import json; d=json.load(open('$O/ab.json')); print('$rep $c $v', d['value'], {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','tree','verify','check','decode')})"
    done
  done
done
echo ok
