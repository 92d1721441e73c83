#!/bin/bash
# rocprofv3 evidence for the bench workload (run ON the GPU box via gpurun).
#   tools/profile.sh <tag> [bench args...]
# Writes gpurun_out/prof_<tag>/: kernel-trace stats, then one PMC pass per
# counter group (separate runs, --pmc never combined with other tracing).
set -euo pipefail
TAG=${1:-r01}; shift || true
ARGS=${*:---steps 3 --warmup 1 --no-cpu-baseline}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" $ARGS > "$OUT/trace.log" 2>&1
pass() {  # pass <name> <counters...>
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- \
        python3 "$ROOT/bench.py" $ARGS > "$OUT/$name.log" 2>&1
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE
pass sq2 SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
pass fetch FETCH_SIZE
pass write WRITE_SIZE
echo "profile $TAG done"
