set -o pipefail
mkdir -p gpurun_out/r02ah
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "host" > gpurun_out/r02ah/test.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r02ah/test.log; exit 1; }
tail -1 gpurun_out/r02ah/test.log
for gb in 64 128 256 512 1024 0; do RBC_GATHER_BLOCKS=$gb timeout -k 10 200 python tools/host_bench.py --pinned --batches 16 --inflight 2 > gpurun_out/r02ah/hb_gb$gb.json 2>&1 || { echo HBFAIL; exit 1; }; done
RBC_HOST_ZERO_COPY=0 timeout -k 10 200 python tools/host_bench.py --pinned --batches 16 --inflight 2 > gpurun_out/r02ah/hb_nozc.json 2>&1 || exit 1
for f in gpurun_out/r02ah/hb_*.json; do echo $f $(grep -o '"interpolate_GBps": [0-9.]*' $f); done
