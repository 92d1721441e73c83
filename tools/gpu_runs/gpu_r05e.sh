# Round 5: validate-lane sweep over client threads, max_wait and arena size at
# 88,064 outstanding (C2), with the host's memcpy-into-pinned ceiling.
set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
for T in 8 16 32; do
  for W in 200 1000; do
    timeout -k 10 120 tools/batcher_bench validate-sweep 256 $T $W 88064 > $O/t${T}_w${W}.jsonl 2>&1 || { echo FAIL $T $W; tail $O/t${T}_w${W}.jsonl; exit 1; }
    echo "T=$T W=$W"; grep -E "copy_ceiling|validate" $O/t${T}_w${W}.jsonl
  done
done
for MB in 64 1024; do
  RBC_BB_ARENA_MB=$MB timeout -k 10 120 tools/batcher_bench validate-sweep 256 16 200 8192 88064 > $O/mb$MB.jsonl 2>&1 || { echo FAIL mb $MB; exit 1; }
  echo "arena $MB MB"; grep validate $O/mb$MB.jsonl
done
echo ok
