set -o pipefail
mkdir -p gpurun_out/r02bc
timeout -k 10 400 python -u -m pytest tests/test_gpu_protocol.py tests/test_gpu_protocol_lockstep.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "batcher or protocol or lockstep or host" > gpurun_out/r02bc/test.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r02bc/test.log; exit 1; }
tail -1 gpurun_out/r02bc/test.log
timeout -k 10 120 ./tests/cpp/rbc_test > gpurun_out/r02bc/cpp.log 2>&1 || { echo CPPFAIL; tail gpurun_out/r02bc/cpp.log; exit 1; }
for a in "128 42 65536 3000 1" "128 42 65536 3000 8" "128 42 65536 3000 16"; do
  timeout -k 10 300 ./tools/protocol_bench $a > gpurun_out/r02bc/p.json 2>&1 || { echo FAIL; cat gpurun_out/r02bc/p.json; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/r02bc/p.json')); print(d['threads'], d['seconds'], d['gpu_launches'], d['bad'], d['thread_seconds'])"
done
timeout -k 10 200 ./tools/batcher_bench 1024 16 64 64 2048 200 | cut -c1-250
