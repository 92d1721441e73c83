# Round 4: the other configs with the node-reuse recheck and the dwordx4 / x3
# gf_regen stores; PMC traffic per kernel at C2 and C4 (pipelined schedule:
# the receive step's kernels, each dispatch alone under --pmc); an A/B of
# merkle_path_kernel's resident blocks per CU (dynamic LDS pad) against its
# branch re-reads at C4.
set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
Q="--no-cpu-baseline --no-pcie"
for cfg in c4 c1 c3; do
  timeout -k 10 300 python bench.py --config $cfg --steps 60 $Q > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { echo BENCHFAIL $cfg; tail -20 $O/bench_$cfg.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$cfg.json')); print('$cfg', d['value'], d['ms_per_step'], d['decoded_ok'], d['values_ok'], d['stage_ms'])"
done
for v in pad20k pad8k; do
  RBC_GPU_LIB=ab/librbc_gpu_$v.so timeout -k 10 300 python bench.py --config c4 --steps 60 $Q > $O/bench_c4_$v.json 2> $O/bench_c4_$v.err || { echo BENCHFAIL $v; tail -20 $O/bench_c4_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_c4_$v.json')); print('c4 $v', d['value'], d['decoded_ok'], d['values_ok'], d['library'], d['stage_ms'])"
done
timeout -k 10 200 python bench.py --config c4 --steps 60 $Q > $O/bench_c4_again.json 2> /dev/null && python -c "import json; d=json.load(open('$O/bench_c4_again.json')); print('c4 again', d['value'])"
bash tools/pmc_passes.sh r04b_c2 --steps 5 --warmup 3 --no-isolated $Q || { echo PMCFAIL c2; exit 1; }
bash tools/pmc_passes.sh r04b_c4 --config c4 --steps 5 --warmup 3 --no-isolated $Q || { echo PMCFAIL c4; exit 1; }
RBC_GPU_LIB=ab/librbc_gpu_pad20k.so bash tools/pmc_passes.sh r04b_c4pad --config c4 --steps 5 --warmup 3 --no-isolated $Q || { echo PMCFAIL pad; exit 1; }
echo ok
