set -o pipefail
mkdir -p gpurun_out/r02ai
cd /tmp && export TMPDIR=/tmp
RBC_GATHER_BLOCKS=64 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $GRAFT_REPO_ROOT/gpurun_out/r02ai/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/host_bench.py --pinned --batches 8 --inflight 2 > $GRAFT_REPO_ROOT/gpurun_out/r02ai/hb.json 2>&1 || exit 1
echo ok
