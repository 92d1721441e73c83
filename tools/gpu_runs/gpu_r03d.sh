# Round 3: GF decode kernels (scalar row offsets, double-buffered loads) --
# parity first, then chunk-size A/B (serial kernel traces + pipelined bench),
# then the r03c runs (configs, priority A/B, profile of the default).
set -o pipefail
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_encoder.py -m gpu --maxfail=3 -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo PARITYFAIL; grep -E "FAILED|Error" $O/parity.log | tail -20; exit 1; }
tail -1 $O/parity.log
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
Q="--no-cpu-baseline --no-pcie --no-isolated --oracle-samples 2"
for v in base src8 src16; do
  lib=""; [ $v != base ] && lib=$R/ab/librbc_gpu_$v.so
  RBC_GPU_LIB_AB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/t4_$v -o run --output-format csv -- python3 $R/bench.py --config c4 --pipeline 0 --steps 5 --warmup 2 $Q > $R/$O/t4_$v.json 2> $R/$O/t4_$v.log || { echo "T4FAIL $v"; exit 1; }
  grep -h "gf_short" $R/$O/t4_$v/run_kernel_stats.csv | cut -d, -f1-4 | sed "s/^/$v /"
done
for v in base lrc12 lrc16; do
  lib=""; [ $v != base ] && lib=$R/ab/librbc_gpu_$v.so
  RBC_GPU_LIB_AB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/t2_$v -o run --output-format csv -- python3 $R/bench.py --config c2 --pipeline 0 --steps 5 --warmup 2 $Q > $R/$O/t2_$v.json 2> $R/$O/t2_$v.log || { echo "T2FAIL $v"; exit 1; }
  grep -h "gf_rows" $R/$O/t2_$v/run_kernel_stats.csv | cut -d, -f1-4 | sed "s/^/$v /"
done
cd $R
B="--no-cpu-baseline --no-pcie --steps 40"
run() {  # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py $B "$@" > $O/$tag.json 2>> $O/runs.err || { echo "RUNFAIL $tag"; tail -20 $O/runs.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['ms_per_step'], {k: round(v, 3) for k, v in d['stage_ms'].items()})"
}
for v in src8 src16; do RBC_GPU_LIB_AB=$R/ab/librbc_gpu_$v.so run c4_$v --config c4; done
for v in lrc12 lrc16; do RBC_GPU_LIB_AB=$R/ab/librbc_gpu_$v.so run c2_$v; done
run c2_base
for c in c1 c3 c4; do run cfg_$c --config $c; done
run c4_fp --config c4 --faults-on proposer
for p in 0,0 0,1 0,3 1,2 2,2 0,2; do run prio_${p/,/_} --wave-prio $p; done
echo ok
