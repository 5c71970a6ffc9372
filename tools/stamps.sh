set -u
for cfg in "1 11" "0,1 8" "0 8" "0,1 12"; do
  set -- $cfg
  MURR_DEBUG_DECODE=$2 timeout -k 10 120 python bench.py --steps 1 --warmup 0 --no-cpu --proj $1 > gpurun_out/st.log 2>gpurun_out/st.err || exit $?
  echo "proj=$1 dbg=$2: $(tail -1 gpurun_out/st.err)"
done
