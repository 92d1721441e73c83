#!/bin/bash
# Round 4: C1 (N = 64, 0.89x of C2 per byte) -- kernel trace + VALU
# instruction counts of the pipelined step, and each kernel's loaded clock
# alone (serial schedule), to price its issue like C2 / C4.
set -o pipefail
Q="--no-cpu-baseline --no-pcie --no-joined-leg"
PASSES="sq1" bash tools/pmc_passes.sh r04q_c1 --config c1 --steps 5 --warmup 3 --no-isolated $Q || { echo PMCFAIL c1; exit 1; }
PASSES="sq1 sq2" bash tools/pmc_passes.sh r04q_c1s --config c1 --pipeline 0 --steps 5 --warmup 3 --no-isolated $Q || { echo PMCFAIL c1s; exit 1; }
echo ok
