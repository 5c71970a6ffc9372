set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_table.py -x -q --timeout 120 --timeout-method thread > gpurun_out/res_tests.log 2>&1; rc=$?; tail -15 gpurun_out/res_tests.log; [ $rc -eq 0 ] || exit $rc
for k in 1000 100000 1000000; do timeout -k 10 120 python bench.py --mode resident --keys $k --steps 30 --warmup 5 > gpurun_out/res_$k.log 2>&1 || exit $?; tail -1 gpurun_out/res_$k.log; done
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/resprof -o res -- python3 $GRAFT_REPO_ROOT/bench.py --mode resident --keys 1000 --steps 20 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/resprof.log 2>&1 || exit $?
find $GRAFT_REPO_ROOT/gpurun_out/resprof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-140
