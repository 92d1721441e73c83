# Round 6, final tree: GPU suite + smoke, the evidence run (gpu_r06j.sh), then
# PMC traffic passes in the joined form at C2, C4, C1 (-> profiles/pmc_traffic_r06ae_*.json
# through tools/pmc_summary.py --value-form joined).
set -o pipefail
RUN=${RUN:-r06ae}
RUN=$RUN bash tools/gpu_runs/gpu_r06i.sh || exit 1
RUN=$RUN bash tools/gpu_runs/gpu_r06j.sh || exit 1
Q="--no-cpu-baseline --no-pcie --no-batcher --no-isolated --no-second-form"
for cfg in c2 c4 c1; do
  PASSES="sq1 fetch write" timeout -k 10 400 bash tools/pmc_passes.sh ${RUN}_$cfg --config $cfg --steps 25 --warmup 3 $Q || { echo PMCFAIL $cfg; exit 1; }
done
echo ok
