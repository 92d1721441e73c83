# Round 3: gf_regen with NW waves per block (3 for short rows: 48 rows per pass)
# and an even group split -- parity (new: exact missing-row counts), FETCH_SIZE / WRITE_SIZE of the
# GF kernel alone (serial, PMC serialises dispatches) at C2 / C4 for this build
# and the previous one (ab/librbc_gpu_regen1.so), then interleaved benches.
set -o pipefail
O=gpurun_out/r03o; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py > $O/parity.log 2>&1 || { echo PARITYFAIL; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
cd /tmp && export TMPDIR=/tmp
Q="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2 --pipeline 0 --steps 3 --warmup 1"
for v in new regen1; do
  lib=""; [ $v != new ] && lib=$R/ab/librbc_gpu_$v.so
  for c in c2 c4; do
    for pc in FETCH_SIZE WRITE_SIZE; do
      RBC_GPU_LIB_AB=$lib timeout -s KILL 120 rocprofv3 --pmc $pc -d $R/$O/p_${c}_${v}_$pc -o run --output-format csv -- python3 $R/bench.py --config $c $Q > /dev/null 2> $R/$O/p.log || { echo "PFAIL $v $c $pc"; tail -5 $R/$O/p.log; exit 1; }
    done
    python3 - <<PY
import csv, collections
for pc in ("FETCH_SIZE", "WRITE_SIZE"):
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open("$R/$O/p_${c}_${v}_" + pc + "/run_counter_collection.csv")):
        if "gf_" in r["Kernel_Name"]:
            acc[r["Dispatch_Id"]] += float(r["Counter_Value"])
    vals = list(acc.values())[-3:]
    print("$c $v", pc, "KiB per launch", [round(x) for x in vals])
PY
  done
done
cd $R
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2 --steps 60"
for rep in 1 2; do
  for c in c2 c1 c4; do
    for v in new regen1; do
      lib=""; [ $v != new ] && lib=$R/ab/librbc_gpu_$v.so
      RBC_GPU_LIB_AB=$lib timeout -k 10 200 python bench.py $B --config $c > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $c $v"; tail -20 $O/ab.err; exit 1; }
      python -c "import json; d=json.load(open('$O/ab.json')); print('$rep $c $v', d['value'], {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','verify','check','decode')})"
    done
  done
done
echo ok
