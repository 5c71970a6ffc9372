set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_table.py -x -q --timeout 120 --timeout-method thread > gpurun_out/enc_tests.log 2>&1; rc=$?; tail -3 gpurun_out/enc_tests.log; [ $rc -le 1 ] || exit $rc
for c in E B C; do timeout -k 10 120 python bench.py --mode encode --enc-config $c --steps 20 --warmup 3 --no-cpu > gpurun_out/enc_$c.log 2>&1 || exit $?; tail -1 gpurun_out/enc_$c.log; done
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/encprof -o enc -- python3 $GRAFT_REPO_ROOT/bench.py --mode encode --enc-config B --steps 10 --warmup 2 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/encprof.log 2>&1 || exit $?
find $GRAFT_REPO_ROOT/gpurun_out/encprof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-160
