set -o pipefail
mkdir -p gpurun_out/r02d
for inf in 1 2 3 4; do
  for pin in "" "--pinned"; do
    RBC_HOST_SLOTS=$inf timeout -k 10 120 python tools/host_bench.py --inflight $inf --batches 12 $pin >> gpurun_out/r02d/host.jsonl 2>>gpurun_out/r02d/host.err || { echo FAIL $inf $pin; tail gpurun_out/r02d/host.err; exit 1; }
  done
done
cat gpurun_out/r02d/host.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); c=d['config']; print(c['inflight'], c['pinned'], d['shard_commit_GBps'], d['interpolate_GBps'])"
