export MURR_DECODE_VERBOSE=1 MURR_JIT_DEFS=MJ_STAMPS
for a in "--config C --blocks 10" "--config D"; do
  timeout -k 10 120 python3 bench.py $a --steps 3 --warmup 1 --no-cpu 2>&1 | grep -E "stamps|decode launch" | sort | uniq -c | tail -4
done
unset MURR_JIT_DEFS
bash tools/perf_quick.sh
