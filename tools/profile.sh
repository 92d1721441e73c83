#!/bin/bash
# rocprofv3 evidence for the bench workload (run ON the GPU box via gpurun).
#   tools/profile.sh <tag> [bench args...]
# Writes gpurun_out/prof_<tag>/: a kernel-trace + stats run of the bench
# command, then one PMC pass per counter group (separate runs; --pmc is never
# combined with other tracing).  Default command = the driver's bench line.
set -euo pipefail
TAG=${1:-r02}; shift || true
ARGS=${*:---steps 20 --warmup 3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" $ARGS > "$OUT/trace.json" 2> "$OUT/trace.log"
pass() {  # pass <name> <counters...>
    local name=$1; shift
    timeout -s KILL 180 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- \
        python3 "$ROOT/bench.py" $ARGS --no-cpu-baseline --no-pcie > "$OUT/$name.json" 2> "$OUT/$name.log"
}
if [ -z "${NO_PMC:-}" ]; then
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE
pass write WRITE_SIZE
fi
echo "profile $TAG done"
