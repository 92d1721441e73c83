set -o pipefail
bash tools/profile.sh r02a || exit 1
python3 tools/pmc_summary.py gpurun_out/prof_r02a --config c2 --last 20 --json gpurun_out/prof_r02a/summary.json --traffic gpurun_out/prof_r02a/pmc_traffic.json > gpurun_out/prof_r02a/summary.txt
python3 tools/trace_summary.py gpurun_out/prof_r02a/trace/run_kernel_trace.csv --config c2 --last 20 --json gpurun_out/prof_r02a/trace_roles.json > gpurun_out/prof_r02a/trace_roles.txt
cat gpurun_out/prof_r02a/trace_roles.txt
