set -o pipefail
mkdir -p gpurun_out/r02y
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $GRAFT_REPO_ROOT/gpurun_out/r02y/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/host_bench.py --pinned --batches 8 --inflight 2 > $GRAFT_REPO_ROOT/gpurun_out/r02y/hb.json 2> $GRAFT_REPO_ROOT/gpurun_out/r02y/hb.err || { echo FAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r02y/hb.err; exit 1; }
cat $GRAFT_REPO_ROOT/gpurun_out/r02y/hb.json
