# receive-step kernel rework (wave-uniform v/r choice, one node body in the walk):
# parity tests, then block size A/B pipelined and standalone
set -o pipefail
O=gpurun_out/r02rx2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "receive_step or verify or interpolate" > $O/test.log 2>&1 || { echo TESTFAIL; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for tpb in 64 256 64 256; do
RBC_RX_TPB=$tpb timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --steps 40 > $O/t$tpb.json 2> $O/t$tpb.err || { echo "FAIL $tpb"; tail -5 $O/t$tpb.err; exit 1; }
python -c "import json; d=json.load(open('$O/t$tpb.json')); print('$tpb', d['value'], d['values_ok'], d['stage_ms'], 'rxstep', d['receive_only']['receive_step']['ms_per_batch'], 'sep', d['receive_only']['ms_per_batch'])"
done
