# Round 5, final tree: the rocprofv3 kernel trace + stats of exactly `python bench.py`.
set -o pipefail
O=gpurun_out/r05x; mkdir -p $O
R=$(pwd)
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof_default -o run --output-format csv -- python3 $R/bench.py > $R/$O/prof_default.json 2> $R/$O/prof_default.err ) || { echo PROFFAIL; tail -20 $O/prof_default.err; exit 1; }
python -c "import json; d=json.load(open('$O/prof_default.json')); print(d['value'], d['roofline']['kernel'], d['roofline']['avg_ms'], d['roofline_encode']['avg_ms'], d['value_joined']['value'])"
echo ok
