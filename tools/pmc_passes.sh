#!/bin/bash
# rocprofv3 counter passes for one bench command (run ON the GPU box via gpurun).
#   tools/pmc_passes.sh <tag> <bench args...>
# Writes gpurun_out/pmc_<tag>/: a kernel-trace + stats run, then one PMC pass
# per counter group, each a separate run (--pmc is never combined with other
# tracing; every group fits the gfx950 slots: <= 8 SQ, <= 4 TCC, <= 2 GRBM).
set -euo pipefail
TAG=$1; shift
ARGS="$*"
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" $ARGS > "$OUT/trace.json" 2> "$OUT/trace.log"
pass() {  # pass <name> <counters...>
    local name=$1; shift
    timeout -s KILL 180 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- \
        python3 "$ROOT/bench.py" $ARGS > "$OUT/$name.json" 2> "$OUT/$name.log"
}
# PASSES (default all): a subset, e.g. PASSES="fetch write" for the traffic alone
want() { [ -z "${PASSES:-}" ] || [[ " $PASSES " == *" $1 "* ]]; }
want sq1 && pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT
want sq2 && pass sq2 SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
want fetch && pass fetch FETCH_SIZE
want write && pass write WRITE_SIZE
echo "pmc $TAG done"
