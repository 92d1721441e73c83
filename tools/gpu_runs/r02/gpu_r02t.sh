set -o pipefail
mkdir -p gpurun_out/r02t
timeout -k 10 600 python -u -m pytest tests/test_gpu_protocol_lockstep.py tests/test_gpu_protocol.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02t/lockstep.log 2>&1 || { echo TESTFAIL; tail -60 gpurun_out/r02t/lockstep.log; exit 1; }
tail -30 gpurun_out/r02t/lockstep.log
