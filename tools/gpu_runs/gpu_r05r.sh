# Round 5 A/B: the N = 256 FFT transforms asked for 3 or 4 waves per SIMD
# (168 / 128 VGPRs, the rest spilled to scratch) against the product's 2
# (250-256 VGPRs): at C4 the receiver's FFT decode runs alone ~0.86 ms a step.
set -o pipefail
O=gpurun_out/r05r; mkdir -p $O
Q="--no-cpu-baseline --no-pcie --no-batcher --no-joined-leg"
line() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['decoded_ok'], d['values_ok'], d['oracle_sample_ok'], d['library'], {k: d['stage_ms'][k] for k in ('enc','leaf','verify','decode')})" "$@"; }
for rep in 1 2; do
  for v in prod wpe3 wpe4; do
    L=""; [ $v != prod ] && L=ab/librbc_gpu_$v.so
    RBC_GPU_LIB=$L timeout -k 10 300 python bench.py --config c4 --steps 60 $Q > $O/c4_${v}_$rep.json 2> $O/c4_${v}_$rep.err || { echo BENCHFAIL $v; tail -20 $O/c4_${v}_$rep.err; exit 1; }
    line $O/c4_${v}_$rep.json c4_${v}_$rep
  done
done
echo ok
