# kernel trace of the bench's receive_step-only pass (and the pipelined steps)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r02rxprof; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-pcie > $O/b.json 2> $O/b.log || { echo FAIL; tail -5 $O/b.log; exit 1; }
echo ok
