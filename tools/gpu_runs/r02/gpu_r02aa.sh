set -o pipefail
mkdir -p gpurun_out/r02aa
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02aa/test.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r02aa/test.log; exit 1; }
tail -2 gpurun_out/r02aa/test.log
for i in 1 2 3; do timeout -k 10 200 python tools/host_bench.py --pinned --batches 12 --inflight $i > gpurun_out/r02aa/hb_pinned_$i.json 2>&1 || { echo HBFAIL; cat gpurun_out/r02aa/hb_pinned_$i.json; exit 1; }; done
timeout -k 10 200 python tools/host_bench.py --batches 12 --inflight 2 > gpurun_out/r02aa/hb_pageable_2.json 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $GRAFT_REPO_ROOT/gpurun_out/r02aa/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/host_bench.py --pinned --batches 8 --inflight 2 > $GRAFT_REPO_ROOT/gpurun_out/r02aa/hb_traced.json 2>&1 || exit 1
cat $GRAFT_REPO_ROOT/gpurun_out/r02aa/hb_*.json
