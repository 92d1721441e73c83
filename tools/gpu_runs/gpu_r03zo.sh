# Round 3, final code: rocprofv3 kernel trace + stats of exactly the driver's
# default command (python bench.py, no arguments), for profiles/.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r03zo; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py > $O/bench.json 2> $O/bench.err || { echo PROFFAIL; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['steps'], d['roofline']['kernel'], d['roofline']['avg_ms'], d['roofline']['frac'])"
echo ok
