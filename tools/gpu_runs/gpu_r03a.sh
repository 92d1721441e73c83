# Round 3, first call: counter evidence for the GF decode at C4 and C2 (serial
# schedule, so each kernel's counters are its own), plus the C4 pipelined trace.
set -o pipefail
O=gpurun_out/r03a; mkdir -p $O
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 4"
timeout -k 10 400 bash tools/pmc_passes.sh r03a_c4s --config c4 --pipeline 0 --steps 5 --warmup 2 $B > $O/c4s.log 2>&1 || { echo C4SFAIL; tail -20 $O/c4s.log; exit 1; }
timeout -k 10 400 bash tools/pmc_passes.sh r03a_c2s --config c2 --pipeline 0 --steps 5 --warmup 2 $B > $O/c2s.log 2>&1 || { echo C2SFAIL; tail -20 $O/c2s.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/c4p -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --config c4 --steps 10 --warmup 3 $B > $GRAFT_REPO_ROOT/$O/c4p.json 2> $GRAFT_REPO_ROOT/$O/c4p.log || { echo C4PFAIL; exit 1; }
echo ok
