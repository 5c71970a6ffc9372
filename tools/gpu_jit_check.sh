set -u
mkdir -p gpurun_out
export MURR_DECODE_VERBOSE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_auto.log 2>&1; rc=$?; echo "auto rc=$rc"; tail -5 gpurun_out/t_auto.log
[ $rc -le 1 ] || exit $rc
MURR_DECODE_JIT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_table.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_jit.log 2>&1; rc=$?; echo "jit rc=$rc"; tail -15 gpurun_out/t_jit.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/b.log 2> gpurun_out/b.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/b.log; tail -3 gpurun_out/b.err
