# Round 4: merkle_path_kernel A/B at C4 -- one instance per wave with four
# branch levels staged in LDS (product) against two instances per wave (L = 8,
# both instances' hash tasks of a level on one wave's lanes, two levels staged);
# interleaved, then the pair's PMC (VALU, reads).
set -o pipefail
O=gpurun_out/r04g; mkdir -p $O
R=$(pwd)
Q="--no-cpu-baseline --no-pcie --no-joined-leg"
for rep in 1 2 3; do
  for v in base pair; do
    if [ $v = base ]; then L=""; else L=$R/ab/librbc_gpu_$v.so; fi
    RBC_GPU_LIB=$L timeout -k 10 300 python bench.py --config c4 --steps 60 $Q > $O/c4_${v}_$rep.json 2> $O/c4_${v}_$rep.err || { echo BENCHFAIL $v; tail -20 $O/c4_${v}_$rep.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['decoded_ok'], d['values_ok'], d['oracle_sample_ok'], d['stage_ms'])" $O/c4_${v}_$rep.json "c4 $v"
  done
done
RBC_GPU_LIB=$R/ab/librbc_gpu_pair.so PASSES="sq1 fetch" bash tools/pmc_passes.sh r04g_c4pair --config c4 --steps 5 --warmup 3 --no-isolated $Q || { echo PMCFAIL; exit 1; }
echo ok
