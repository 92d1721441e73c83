# Round 3: rocprof evidence of the new default (trace + PMC), per-config runs,
# wave-priority and fault-placement A/B.
set -o pipefail
O=gpurun_out/r03c; mkdir -p $O
B="--no-cpu-baseline --no-pcie --steps 40"
run() {  # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py $B "$@" > $O/$tag.json 2>> $O/runs.err || { echo "RUNFAIL $tag"; tail -20 $O/runs.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['ms_per_step'], {k: round(v, 3) for k, v in d['stage_ms'].items()})"
}
for c in c1 c3 c4; do run cfg_$c --config $c; done
run c4_fp --config c4 --faults-on proposer
run c4_join --config c4 --join
for p in 0,0 0,1 0,3 1,2 2,2 0,2; do run prio_${p/,/_} --wave-prio $p; done
timeout -k 10 900 bash tools/profile.sh r03 > $O/profile.log 2>&1 || { echo PROFFAIL; tail -30 $O/profile.log; exit 1; }
echo ok
