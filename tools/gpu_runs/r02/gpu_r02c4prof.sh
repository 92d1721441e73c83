# kernel trace of the C4 bench (N=256, 64 KiB, 16,384 instances) under the default schedule
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r02c4prof; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline --no-pcie > $O/b.json 2> $O/b.log || { echo FAIL; tail -5 $O/b.log; exit 1; }
echo ok
