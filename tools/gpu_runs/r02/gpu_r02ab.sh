set -o pipefail
mkdir -p gpurun_out/r02ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02ab/test.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r02ab/test.log; exit 1; }
tail -2 gpurun_out/r02ab/test.log
for i in 1 2 3; do timeout -k 10 200 python tools/host_bench.py --pinned --batches 16 --inflight $i > gpurun_out/r02ab/hb_pinned_$i.json 2>&1 || { echo HBFAIL; cat gpurun_out/r02ab/hb_pinned_$i.json; exit 1; }; done
timeout -k 10 200 python tools/host_bench.py --batches 12 --inflight 2 > gpurun_out/r02ab/hb_pageable_2.json 2>&1 || exit 1
for f in gpurun_out/r02ab/hb_*.json; do echo $f; cat $f; done
