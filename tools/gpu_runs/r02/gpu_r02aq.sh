set -o pipefail
mkdir -p gpurun_out/r02aq
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02aq/test.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r02aq/test.log; exit 1; }
tail -1 gpurun_out/r02aq/test.log
timeout -k 10 200 ./tools/batcher_bench 1024 16 64 64 2048 200 > gpurun_out/r02aq/batcher.jsonl 2>&1 || { echo FAIL; cat gpurun_out/r02aq/batcher.jsonl; exit 1; }
for i in 1 2 3 4; do timeout -k 10 200 python tools/host_bench.py --pinned --batches 16 --inflight $i > gpurun_out/r02aq/hb_$i.json 2>&1 || { echo HBFAIL; exit 1; }; done
cat gpurun_out/r02aq/batcher.jsonl | cut -c1-300
for i in 1 2 3 4; do grep -o '"inflight": [0-9]*\|"shard_commit_GBps": [0-9.]*\|"interpolate_GBps": [0-9.]*\|"shard_commit_val_msg_GBps": [0-9.]*' gpurun_out/r02aq/hb_$i.json | tr '\n' ' '; echo; done
