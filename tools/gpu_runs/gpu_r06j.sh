# Round 6, final tree (2/2): the default bench line twice, the rocprofv3 kernel
# trace + stats of exactly `python bench.py`, the other configs' lines, and a
# 2-rank rehearsal with the host-fed leg on both ranks.
set -o pipefail
O=gpurun_out/${RUN:-r06j}; mkdir -p $O
R=$(pwd)
for rep in 1 2; do
  t0=$(date +%s.%N)
  timeout -k 10 600 python bench.py > $O/bench_default_$rep.json 2> $O/bench_default_$rep.err || { echo BENCHFAIL; tail -30 $O/bench_default_$rep.err; exit 1; }
  python -c "import time; print('wall', round(time.time() - $t0, 1), 's')"
  python -c "import json; d=json.load(open('$O/bench_default_$rep.json')); p=d['pcie_inclusive']; b=d['batcher']; print('value', d['value'], d['ms_per_step'], 'row', d['value_row_view']['value'], 'host', p['aggregate_GBps'], 'fused', p['fused']['aggregate_GBps'], 'epoch', b['epoch']['GBps'], b['epoch']['GBps_full_rehash'], 'sweep', [x['GBps'] for x in b['sweep']], 'cpu', d['cpu_baseline']['value'], 'frac', d['roofline']['frac'], d['roofline']['traffic'])"
done
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof_default -o run --output-format csv -- python3 $R/bench.py > $R/$O/prof_default.json 2> $R/$O/prof_default.err ) || { echo PROFFAIL; tail -20 $O/prof_default.err; exit 1; }
python -c "import json; d=json.load(open('$O/prof_default.json')); print('profiled', d['value'], d['roofline']['kernel'], d['roofline']['avg_ms'])"
for cfg in c1 c3 c4; do
  timeout -k 10 600 python bench.py --config $cfg --no-cpu-baseline > $O/$cfg.json 2> $O/$cfg.err || { echo BENCHFAIL $cfg; tail -30 $O/$cfg.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$cfg.json')); p=d['pcie_inclusive']; print('$cfg', d['value'], d['ms_per_step'], 'row', d['value_row_view']['value'], 'host', p['aggregate_GBps'], 'fused', p['fused']['aggregate_GBps'])"
done
timeout -k 10 600 python bench.py --gpus 2 --rehearse-on-one-gpu --no-cpu-baseline --no-batcher > $O/rehearse2.json 2> $O/rehearse2.err || { echo BENCHFAIL r2; tail -30 $O/rehearse2.err; exit 1; }
python -c "import json; d=json.load(open('$O/rehearse2.json')); p=d['pcie_inclusive']; print('2-rank rehearsal', d['value'], 'host', p['aggregate_GBps'], p['per_rank_GBps'], 'fused', p['fused']['aggregate_GBps'], p['fused']['per_rank_GBps'], p['ok'])"
echo ok
