# rocprof kernel stats of the final code at C1, C3 (1,024 per GPU) and C4
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r02cfgprof; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in c1 c3 c4; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$c -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-pcie > $O/$c.json 2> $O/$c.log || { echo "FAIL $c"; tail -5 $O/$c.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/$c.json')); print('$c', d['value'], d['values_ok'], d['oracle_sample_ok'])"
done
