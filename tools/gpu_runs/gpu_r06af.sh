# Round 6: the C4 host-fed epoch's kernel + copy trace after the value repack
# and the short-row gathers (compare profiles/r06ac/).
set -o pipefail
O=gpurun_out/${RUN:-r06af}; mkdir -p $O
R=$(pwd)
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/tools/host_bench.py --config c4 --epoch 16384 > $R/$O/host_c4_prof.json 2> $R/$O/host_c4_prof.err ) || { echo PROFFAIL; tail -20 $O/host_c4_prof.err; exit 1; }
python -c "import json; d=json.load(open('$O/host_c4_prof.json')); print('drop-in', d['GBps'], 'kept', d['kept']['GBps'], 'fused', d['fused']['GBps'], d['alone_GBps'])"
head -12 $O/prof/run_kernel_stats.csv | cut -c1-200
head -6 $O/prof/run_memory_copy_stats.csv

T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_gpu_verified.py tests/test_gpu_batcher.py tests/test_gpu_protocol.py > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo ok
