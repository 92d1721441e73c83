# Round 6: the join split by row length -- join parity and C4 bench tests,
# PMC traffic at C4 on this tree (the decode no longer writes the joined
# value there), then the C4 line twice and the C2 line once.
set -o pipefail
O=gpurun_out/${RUN:-r06an}; mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 900 $T tests/test_gpu_parity.py tests/test_gpu_bench.py -k "fused_join or row_view or c4 or join" > $O/tests.txt 2>&1 || { echo TESTFAIL; tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
Q="--no-cpu-baseline --no-pcie --no-batcher --no-isolated --no-second-form"
PASSES="sq1 fetch write" timeout -k 10 400 bash tools/pmc_passes.sh r06an_c4 --config c4 --steps 25 --warmup 3 $Q || { echo PMCFAIL; exit 1; }
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $O/c4_$rep.json 2> $O/c4_$rep.err || { echo BENCHFAIL; tail -20 $O/c4_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_$rep.json')); print('c4', d['value'], d['ms_per_step'], 'row', d['value_row_view']['value'], d['stage_ms']['decode'], d['values_ok'], d['pcie_inclusive']['aggregate_GBps'], d['pcie_inclusive']['fused']['aggregate_GBps'])"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-batcher --no-pcie > $O/c2.json 2> $O/c2.err || { echo BENCHFAIL; tail -20 $O/c2.err; exit 1; }
python -c "import json; d=json.load(open('$O/c2.json')); print('c2', d['value'], d['ms_per_step'], 'row', d['value_row_view']['value'])"
echo ok
