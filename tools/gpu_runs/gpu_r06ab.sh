# Round 6: the host-fed epoch (C2, 1,024 instances) against its sub-batch
# size and submissions in flight per side: drop-in calls, kept rows, fused.
set -o pipefail
O=gpurun_out/${RUN:-r06ab}; mkdir -p $O
for cfg in "64 2" "128 2" "256 2" "64 3" "128 3" "32 4"; do
  set -- $cfg
  timeout -k 10 300 python tools/host_bench.py --epoch 1024 --sub $1 --inflight $2 > $O/host_s$1_i$2.json 2> $O/host_s$1_i$2.err || { echo HOSTFAIL $cfg; tail -20 $O/host_s$1_i$2.err; exit 1; }
  python -c "import json; d=json.load(open('$O/host_s$1_i$2.json')); print('sub $1 inflight $2', 'drop-in', d['GBps'], 'kept', d['kept']['GBps'], 'fused', d['fused']['GBps'], d['ok'])"
done
echo ok
