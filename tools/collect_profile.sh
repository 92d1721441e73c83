#!/bin/bash
# Copy the judged evidence of a tools/profile.sh run into profiles/ (run HERE,
# after gpurun merged gpurun_out/prof_<tag>):
#   tools/collect_profile.sh <tag> [--config c2] [--instances 1024]
# -> profiles/<tag>_kernel_stats.csv      rocprofv3 --stats of the bench command
#    profiles/<tag>_trace_roles.{txt,json} per-role averages over the timed launches
#    profiles/<tag>_pmc_summary.json       per-role PMC (SQ pass, FETCH_SIZE, WRITE_SIZE)
#    profiles/pmc_traffic_<tag>.json       HBM bytes per launch, read by bench.py (roofline.traffic)
#    profiles/<tag>_profiled_bench.json    the bench line of the traced run
set -euo pipefail
TAG=$1; shift
CFG=c2; INST=1024
while [ $# -gt 0 ]; do
    case $1 in
        --config) CFG=$2; shift 2 ;;
        --instances) INST=$2; shift 2 ;;
        *) echo "unknown $1"; exit 2 ;;
    esac
done
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/gpurun_out/prof_$TAG
P=$ROOT/profiles
cp "$D/trace/run_kernel_stats.csv" "$P/${TAG}_kernel_stats.csv"
python3 "$ROOT/tools/trace_summary.py" "$D/trace/run_kernel_trace.csv" --config "$CFG" --instances "$INST" --last 20 \
    --json "$P/${TAG}_trace_roles.json" > "$P/${TAG}_trace_roles.txt"
python3 "$ROOT/tools/pmc_summary.py" "$D" --config "$CFG" --instances "$INST" --last 20 \
    --json "$P/${TAG}_pmc_summary.json" --traffic "$P/pmc_traffic_${TAG}.json" > /dev/null
cp "$D/trace.json" "$P/${TAG}_profiled_bench.json"
echo "collected $TAG into profiles/"
