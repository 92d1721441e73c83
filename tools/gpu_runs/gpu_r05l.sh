# Round 5: PMC traffic (FETCH_SIZE, WRITE_SIZE) + kernel traces at C3, as the
# bench runs it (1,024 x 4 MiB per GPU, pipelined) and as configs[3] states it
# (all 8,192 x 4 MiB on one GPU, serial) -> profiles/pmc_traffic_r05l_c3*.json,
# so the C3 lines' rooflines carry measured traffic too.
set -o pipefail
Q="--no-cpu-baseline --no-pcie --no-isolated --no-joined-leg --no-batcher"
PASSES="fetch write" timeout -k 10 500 bash tools/pmc_passes.sh r05l_c3 --config c3 --steps 25 --warmup 3 $Q || { echo PMCFAIL c3; exit 1; }
PASSES="fetch write" timeout -k 10 600 bash tools/pmc_passes.sh r05l_c3_8192 --config c3 --total-instances 8192 --steps 3 --warmup 1 $Q || { echo PMCFAIL c3_8192; exit 1; }
echo ok
