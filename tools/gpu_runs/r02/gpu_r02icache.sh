# Instruction-cache counters per kernel: pipelined default vs serial schedule
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r02icache; mkdir -p $O
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for sched in 1 0; do
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU -d $O/p$sched -o run --output-format csv -- \
    python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie --no-isolated --pipeline $sched > $O/p$sched.json 2> $O/p$sched.log || { echo "FAIL pmc $sched"; tail -5 $O/p$sched.log; exit 1; }
done
echo icache done
