# Round 3: gf_regen under the pipeline -- the decode kernels' issue priority
# and the GF kernel's occupancy (A/B builds from tools/build_ab.sh), C2 / C1 /
# C4, interleaved, against the committed library (ab/librbc_gpu_r03base.so).
set -o pipefail
O=gpurun_out/r03j; mkdir -p $O
R=$GRAFT_REPO_ROOT
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2 --steps 60"
for rep in 1 2; do
  for c in c2 c1 c4; do
    for v in new r03base gfp1 gfp0 decp1 decp0 wpe2; do
      lib=""; [ $v != new ] && lib=$R/ab/librbc_gpu_$v.so
      RBC_GPU_LIB_AB=$lib timeout -k 10 200 python bench.py $B --config $c > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $c $v"; tail -20 $O/ab.err; exit 1; }
      python -c "import json; d=json.load(open('$O/ab.json')); print('$rep $c $v', d['value'], {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','verify','check','decode')})"
    done
  done
done
echo ok
