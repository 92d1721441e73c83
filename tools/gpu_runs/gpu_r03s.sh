# Round 3: gf_regen table build with row-major lanes (no LDS bank conflicts on
# the table stores) vs the previous build (ab/librbc_gpu_regen2.so): parity,
# SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS of the GF kernel alone, interleaved benches.
set -o pipefail
O=gpurun_out/r03s; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py > $O/parity.log 2>&1 || { echo PARITYFAIL; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
cd /tmp && export TMPDIR=/tmp
Q="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2 --pipeline 0 --steps 3 --warmup 1"
for v in new regen2; do
  lib=""; [ $v != new ] && lib=$R/ab/librbc_gpu_$v.so
  for c in c2 c4; do
    RBC_GPU_LIB_AB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES -d $R/$O/p_${c}_$v -o run --output-format csv -- python3 $R/bench.py --config $c $Q > /dev/null 2> $R/$O/p.log || { echo "PFAIL $v $c"; tail -5 $R/$O/p.log; exit 1; }
    python3 - <<PY
import csv, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open("$R/$O/p_${c}_$v/run_counter_collection.csv")):
    if "gf_regen" in r["Kernel_Name"]:
        acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
last = list(acc.values())[-1]
print("$c $v", {k: round(x / 1e6, 2) for k, x in last.items()})
PY
  done
done
cd $R
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2 --steps 60"
for rep in 1 2 3; do
  for c in c2 c1 c4; do
    for v in new regen2; do
      lib=""; [ $v != new ] && lib=$R/ab/librbc_gpu_$v.so
      RBC_GPU_LIB_AB=$lib timeout -k 10 200 python bench.py $B --config $c > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $c $v"; tail -20 $O/ab.err; exit 1; }
      python -c "import json; d=json.load(open('$O/ab.json')); print('$rep $c $v', d['value'], {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','verify','check','decode')})"
    done
  done
done
echo ok
