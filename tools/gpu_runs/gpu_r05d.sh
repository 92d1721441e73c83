# Round 5: the validate lane (lock-light reservation, launcher + completer)
# then the PMC / trace evidence at C1, C2, C4 (gpu_r05b.sh).
set -o pipefail
bash tools/gpu_runs/gpu_r05c.sh || exit 1
bash tools/gpu_runs/gpu_r05b.sh || exit 1
