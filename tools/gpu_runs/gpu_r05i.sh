# Round 5: blocking-sync slot events and target-size sealing; the validate
# lane's CPU use (bash `times`) and client-thread count at 8,192 / 88,064 outstanding.
set -o pipefail
O=gpurun_out/r05i; mkdir -p $O
for T in 8 12 16; do
  ( TIMEFORMAT="T=$T wall %R s user %U s sys %S s"; time timeout -k 10 120 tools/batcher_bench validate-sweep 256 $T 200 8192 88064 > $O/t$T.jsonl 2> $O/t$T.err ) 2>&1 || { echo FAIL $T; tail $O/t$T.err; exit 1; }
  grep -E "copy_ceiling|validate" $O/t$T.jsonl | cut -c1-250
done
echo ok
