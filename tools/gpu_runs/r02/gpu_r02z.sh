set -o pipefail
mkdir -p gpurun_out/r02z
timeout -k 10 200 python tools/host_bench.py --pinned --batches 12 --inflight 2 > gpurun_out/r02z/sdma1.json 2>&1 || { echo FAIL; tail gpurun_out/r02z/sdma1.json; exit 1; }
HSA_ENABLE_SDMA=0 timeout -k 10 200 python tools/host_bench.py --pinned --batches 12 --inflight 2 > gpurun_out/r02z/sdma0.json 2>&1 || { echo FAIL; tail gpurun_out/r02z/sdma0.json; exit 1; }
RBC_HOST_SLOTS=3 timeout -k 10 200 python tools/host_bench.py --pinned --batches 12 --inflight 3 > gpurun_out/r02z/slots3.json 2>&1 || { echo FAIL; exit 1; }
cat gpurun_out/r02z/*.json
