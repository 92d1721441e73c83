# Round 4: gf_regen_kernel without scratch spills (the extra HBM writes and
# reads of r04b were its dirty spill lines); the default bench with the
# joined-value leg; C4 / C1; merkle_path_kernel's resident blocks per CU
# (dynamic LDS pad, A/B builds) interleaved with the default; PMC traffic.
set -o pipefail
O=gpurun_out/r04c; mkdir -p $O
R=$(pwd)
Q="--no-cpu-baseline --no-pcie"
line() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['decoded_ok'], d['values_ok'], (d.get('value_joined') or {}).get('value'), d['stage_ms'])" "$@"; }
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCHFAIL; tail -20 $O/bench_default.err; exit 1; }
line $O/bench_default.json default
for rep in 1 2; do
  for v in base pad12k pad20k pad28k; do
    if [ $v = base ]; then L=""; else L=$R/ab/librbc_gpu_$v.so; fi
    RBC_GPU_LIB=$L timeout -k 10 300 python bench.py --config c4 --steps 60 --no-joined-leg $Q > $O/c4_${v}_$rep.json 2> $O/c4_${v}_$rep.err || { echo BENCHFAIL $v; tail -20 $O/c4_${v}_$rep.err; exit 1; }
    line $O/c4_${v}_$rep.json "c4 $v"
  done
done
timeout -k 10 300 python bench.py --config c1 --steps 60 --no-joined-leg $Q > $O/c1.json 2> $O/c1.err && line $O/c1.json c1
PASSES="fetch write" bash tools/pmc_passes.sh r04c_c2 --steps 5 --warmup 3 --no-isolated --no-joined-leg $Q || { echo PMCFAIL c2; exit 1; }
PASSES="fetch write" bash tools/pmc_passes.sh r04c_c4 --config c4 --steps 5 --warmup 3 --no-isolated --no-joined-leg $Q || { echo PMCFAIL c4; exit 1; }
RBC_GPU_LIB=$R/ab/librbc_gpu_pad20k.so PASSES="fetch" bash tools/pmc_passes.sh r04c_c4pad20k --config c4 --steps 5 --warmup 3 --no-isolated --no-joined-leg $Q || { echo PMCFAIL pad; exit 1; }
RBC_GPU_LIB=$R/ab/librbc_gpu_pad28k.so PASSES="fetch" bash tools/pmc_passes.sh r04c_c4pad28k --config c4 --steps 5 --warmup 3 --no-isolated --no-joined-leg $Q || { echo PMCFAIL pad; exit 1; }
echo ok
