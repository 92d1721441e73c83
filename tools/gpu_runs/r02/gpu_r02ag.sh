set -o pipefail
mkdir -p gpurun_out/r02ag
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02ag/test.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r02ag/test.log; exit 1; }
tail -2 gpurun_out/r02ag/test.log
for i in 2 3; do timeout -k 10 200 python tools/host_bench.py --pinned --batches 16 --inflight $i > gpurun_out/r02ag/hb_pinned_$i.json 2>&1 || { echo HBFAIL; cat gpurun_out/r02ag/hb_pinned_$i.json; exit 1; }; done
RBC_HOST_ZERO_COPY=0 timeout -k 10 200 python tools/host_bench.py --pinned --batches 16 --inflight 2 > gpurun_out/r02ag/hb_pinned_2_nozc.json 2>&1 || exit 1
for f in gpurun_out/r02ag/hb_*.json; do echo $f; cat $f; done
