# Round 6: PMC + kernel traces at C2, C4, C1 in the joined value form (the
# bench's `value` since round 6; 25 timed steps: >= 20 timed launches per
# role) -> profiles/pmc_traffic_r06h_*.json (tools/pmc_summary.py --value-form joined).
set -o pipefail
Q="--no-cpu-baseline --no-pcie --no-batcher --no-isolated --no-second-form"
for cfg in c2 c4 c1; do
  PASSES="sq1 fetch write" timeout -k 10 400 bash tools/pmc_passes.sh r06h_$cfg --config $cfg --steps 25 --warmup 3 $Q || { echo PMCFAIL $cfg; exit 1; }
done
echo ok
