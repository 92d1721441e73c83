set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r02_c4s/trace -o run --output-format csv -- python3 $R/bench.py --config c4 --steps 10 --warmup 2 --pipeline 0 --no-cpu-baseline --no-pcie > $R/gpurun_out/prof_r02_c4s/bench.json 2>$R/gpurun_out/prof_r02_c4s/bench.err || exit 1
cd $R && python3 tools/trace_summary.py gpurun_out/prof_r02_c4s/trace/run_kernel_trace.csv --config c4 --instances 16384 --last 10
