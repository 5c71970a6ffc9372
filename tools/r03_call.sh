#!/usr/bin/env bash
# Round-3 working call: encode parity tests, encode benches, ceiling probes.
set -u
export TMPDIR=/tmp
out=gpurun_out/r03
mkdir -p $out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 3 "$out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
for s in ${STEPS:-enc_tests enc_bench probes}; do
  case $s in
    enc_tests) step enc_tests 400 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_table.py tests/test_gpu_fullsize.py tests/test_gpu_resident.py tests/test_gpu_scan.py -m gpu -x -q --timeout 120 --timeout-method thread ;;
    enc_bench)
      for c in E B C; do step enc_$c 200 python bench.py --mode encode --enc-config $c --steps 10 --warmup 2; done ;;
    probes)
      step b_direct 200 tools/ubench/b_direct
      step lds_mix2 100 tools/ubench/lds_mix2
      step mix_bw 100 tools/ubench/mix_bw ;;
    bench) step bench 200 python bench.py ;;
    tests) step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
  esac
done
