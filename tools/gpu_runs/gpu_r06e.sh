# Round 6: kernel + memory-copy trace of the host-fed epoch (drop-in calls and
# the fused receive): which copies / kernels overlap on the PCIe link?
set -o pipefail
O=gpurun_out/r06e; mkdir -p $O
R=$(pwd)
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 $R/tools/host_bench.py --epoch 1024 --inflight 2 > $R/$O/host.json 2> $R/$O/host.err ) || { echo PROFFAIL; tail -20 $O/host.err; exit 1; }
python -c "import json; d=json.load(open('$O/host.json')); print(d['GBps'], d['fused']['GBps'], d['ok']); [print(w[0], w[1], w[2]) for w in d['timed_windows_ns']]" > $O/windows.txt
cat $O/windows.txt
tail -2 $O/windows.txt | while read k a b; do python tools/copy_overlap.py $O/trace $a $b | tee $O/overlap_$k.json; done
ls $O/trace/*/ | head
echo ok
