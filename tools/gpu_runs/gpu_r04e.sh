# Round 4: merkle_path_kernel A/B at C4 -- one instance per wave holding 4
# branch levels per leaf (product) against two instances per wave (L = 8:
# the level's hash tasks of both on one wave's lanes) holding 2 or 4 levels;
# interleaved, then each one's merkle_path reads (FETCH_SIZE); and gf_regen with C4's
# 768-B row as one 12-B-per-lane tile per wave (W = 3, every row; A/B regenw3).
set -o pipefail
O=gpurun_out/r04e; mkdir -p $O
R=$(pwd)
Q="--no-cpu-baseline --no-pcie --no-joined-leg"
for rep in 1 2; do
  for v in base pairq2 pairq4 regenw3; do
    if [ $v = base ]; then L=""; else L=$R/ab/librbc_gpu_$v.so; fi
    RBC_GPU_LIB=$L timeout -k 10 300 python bench.py --config c4 --steps 60 $Q > $O/c4_${v}_$rep.json 2> $O/c4_${v}_$rep.err || { echo BENCHFAIL $v; tail -20 $O/c4_${v}_$rep.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['decoded_ok'], d['values_ok'], d['oracle_sample_ok'], d['stage_ms'])" $O/c4_${v}_$rep.json "c4 $v"
  done
done
for v in pairq2 pairq4 regenw3; do
  RBC_GPU_LIB=$R/ab/librbc_gpu_$v.so PASSES="sq1 fetch" bash tools/pmc_passes.sh r04e_c4$v --config c4 --steps 5 --warmup 3 --no-isolated $Q || { echo PMCFAIL $v; exit 1; }
done
echo ok
