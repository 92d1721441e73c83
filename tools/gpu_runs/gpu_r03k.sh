# Round 3: interpolate's GF transforms at the commit side's priority level --
# gf_regen (product) vs the round-2 GF kernels with the same rule
# (ab/librbc_gpu_oldgfdec0.so) vs the committed library (ab/librbc_gpu_r03base.so),
# and commit / receive levels, C2 / C1 / C4, interleaved.
set -o pipefail
O=gpurun_out/r03k; mkdir -p $O
R=$GRAFT_REPO_ROOT
B="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2 --steps 60"
for rep in 1 2; do
  for c in c2 c1 c4; do
    for v in new:0,2 r03base:0,2 oldgfdec0:0,2 new:1,2 new:0,1 new:1,3; do
      lib=${v%%:*}; p=${v##*:}; L=""; [ $lib != new ] && L=$R/ab/librbc_gpu_$lib.so
      RBC_GPU_LIB_AB=$L timeout -k 10 200 python bench.py $B --config $c --wave-prio $p > $O/ab.json 2>> $O/ab.err || { echo "ABFAIL $c $v"; tail -20 $O/ab.err; exit 1; }
      python -c "import json; d=json.load(open('$O/ab.json')); print('$rep $c $v', d['value'], {k: round(v, 2) for k, v in d['stage_ms'].items() if k in ('enc','leaf','verify','check','decode')})"
    done
  done
done
echo ok
