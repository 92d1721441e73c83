# Round 5: the validate lane with one atomic add per reservation (no lock):
# GPU test + sweep, and the client-thread count at 8,192 / 88,064 outstanding.
set -o pipefail
bash tools/gpu_runs/gpu_r05c.sh || exit 1
bash tools/gpu_runs/gpu_r05i.sh || exit 1
