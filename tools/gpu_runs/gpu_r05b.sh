# Round 5: PMC + kernel traces at C1, C2, C4 (25 timed steps: >= 20 timed
# launches per role), and the serial schedule's per-kernel loaded clock at C2
# and C4 -> profiles/pmc_traffic_r05b_*.json, valu_clock_r05b_*.json.
set -o pipefail
Q="--no-cpu-baseline --no-pcie --no-isolated --no-joined-leg"
for cfg in c2 c4 c1; do
  PASSES="sq1 fetch write" timeout -k 10 400 bash tools/pmc_passes.sh r05b_$cfg --config $cfg --steps 25 --warmup 3 $Q || { echo PMCFAIL $cfg; exit 1; }
done
for cfg in c2 c4; do
  PASSES="sq1 sq2" timeout -k 10 300 bash tools/pmc_passes.sh r05b_${cfg}s --config $cfg --pipeline 0 --steps 6 --warmup 2 $Q || { echo PMCFAIL ${cfg}s; exit 1; }
done
echo ok
