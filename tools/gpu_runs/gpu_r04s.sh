#!/bin/bash
# Round 4: C1 traffic passes (FETCH_SIZE, WRITE_SIZE) beside r04q's VALU pass,
# so the C1 line carries PMC traffic and the step's measured VALU issue too.
set -o pipefail
Q="--no-cpu-baseline --no-pcie --no-joined-leg"
PASSES="sq1 fetch write" bash tools/pmc_passes.sh r04s_c1 --config c1 --steps 5 --warmup 3 --no-isolated $Q || { echo PMCFAIL c1; exit 1; }
echo ok
