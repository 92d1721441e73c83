set -o pipefail
mkdir -p gpurun_out/r02am
timeout -k 10 200 ./tools/batcher_bench_old 256 16 64 > gpurun_out/r02am/old.jsonl 2>&1 || { echo OLDFAIL; cat gpurun_out/r02am/old.jsonl; exit 1; }
timeout -k 10 200 ./tools/batcher_bench 256 16 64 > gpurun_out/r02am/new.jsonl 2>&1 || { echo NEWFAIL; cat gpurun_out/r02am/new.jsonl; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_protocol.py tests/test_gpu_protocol_lockstep.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "batcher or protocol or lockstep" > gpurun_out/r02am/test.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r02am/test.log; exit 1; }
tail -1 gpurun_out/r02am/test.log
echo OLD; cat gpurun_out/r02am/old.jsonl; echo NEW; cat gpurun_out/r02am/new.jsonl
