# Round 5: kernel + memory-copy trace of the validate lane at 88,064 outstanding
# (C2 messages): launch sizes, H2D vs kernel overlap across the lane's launches.
set -o pipefail
O=gpurun_out/r05g; mkdir -p $O
R=$(pwd)
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/$O/trace -o run --output-format csv -- $R/tools/batcher_bench validate-sweep 256 16 200 88064 > $R/$O/sweep.jsonl 2> $R/$O/sweep.err ) || { echo PROFFAIL; tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
ls $O/trace
echo ok
