# Round 4: gf_regen_kernel rebuilt column-split (one wave per column tile owns
# every missing row; block-shared LDS tables): GPU suite, default bench, C4 /
# C1, PMC traffic + VALU at C2 / C4; the FETCH_SIZE calibration probe; a
# serial-schedule trace + SQ pass at C2 for per-kernel loaded clocks.
set -o pipefail
O=gpurun_out/r04d; mkdir -p $O
R=$(pwd)
Q="--no-cpu-baseline --no-pcie"
line() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['decoded_ok'], d['values_ok'], (d.get('value_joined') or {}).get('value'), d['stage_ms'])" "$@"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|error|assert" $O/gputest.log | tail -40; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 400 python bench.py --no-pcie > $O/bench_default.json 2> $O/bench_default.err || { echo BENCHFAIL; tail -20 $O/bench_default.err; exit 1; }
line $O/bench_default.json default
for cfg in c4 c1 c2; do
  timeout -k 10 300 python bench.py --config $cfg --steps 60 --no-joined-leg $Q > $O/$cfg.json 2> $O/$cfg.err || { echo BENCHFAIL $cfg; tail -20 $O/$cfg.err; exit 1; }
  line $O/$cfg.json $cfg
done
PASSES="sq1 fetch write" bash tools/pmc_passes.sh r04d_c2 --steps 5 --warmup 3 --no-isolated --no-joined-leg $Q || { echo PMCFAIL c2; exit 1; }
PASSES="sq1 fetch write" bash tools/pmc_passes.sh r04d_c4 --config c4 --steps 5 --warmup 3 --no-isolated --no-joined-leg $Q || { echo PMCFAIL c4; exit 1; }
PASSES="sq1 sq2" bash tools/pmc_passes.sh r04d_c2s --pipeline 0 --steps 5 --warmup 3 --no-isolated --no-joined-leg $Q || { echo PMCFAIL c2s; exit 1; }
mkdir -p $O/calib && cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/$O/calib -o run --output-format csv -- $R/tools/probes/fetch_calib > $R/$O/calib.txt 2>&1 || { echo CALIBFAIL; tail -20 $R/$O/calib.txt; exit 1; }
grep useful $R/$O/calib.txt
cd $R && bash tools/gpu_runs/gpu_r04e.sh || { echo R04EFAIL; exit 1; }
echo ok
