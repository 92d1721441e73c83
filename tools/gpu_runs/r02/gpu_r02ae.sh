set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r02ae
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
A="$GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pcie --no-isolated"
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH -d $OUT/pipe -o run --output-format csv -- python3 $A > $OUT/pipe.json 2> $OUT/pipe.log || { echo FAIL1; tail -5 $OUT/pipe.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH -d $OUT/ser -o run --output-format csv -- python3 $A --pipeline 0 > $OUT/ser.json 2> $OUT/ser.log || { echo FAIL2; tail -5 $OUT/ser.log; exit 1; }
echo ok
