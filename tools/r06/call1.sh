#!/usr/bin/env bash
# Round 6, call 1: the extended window (MJ_XWIN) on config B -- parity tests,
# interleaved A/B with the LDS ablations, and the LDS counter passes.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c1}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 4 "$out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
TL=$PWD/murr_amd/libmurr_codec_tuning.so
run tests 500 "$PY" -u -m pytest tests/test_gpu_decode.py tests/test_gpu_ro32.py tests/test_gpu_bench_launch.py tests/test_gpu_sst.py -m gpu -x -q --timeout 120 --timeout-method thread
run ab 900 "$PY" tools/ab.py --reps 3 \
  --env x0=MURR_LIB=$TL --env x0=MURR_JIT_DEFS=MJ_XWIN=0 \
  --env x1=MURR_LIB=$TL --env x1=MURR_JIT_DEFS=MJ_XWIN=1 \
  --env ldsx0=MURR_LIB=$TL --env ldsx0=MURR_JIT_DEFS=MJ_XWIN=0,MJ_ABL_LDSX=1 \
  --env lo=MURR_LIB=$TL --env lo=MURR_JIT_DEFS=MJ_ABL_LOADONLY=1 \
  "x0::" "x1::" "ldsx0::" "lo::--no-verify"
cp -r gpurun_out/ab $out/ab
for v in "x0:MJ_XWIN=0" "x1:MJ_XWIN=1" "ldsx0:MJ_XWIN=0,MJ_ABL_LDSX=1" "lo:MJ_ABL_LOADONLY=1"; do
  n=${v%%:*}; d=${v#*:}
  i=0
  for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" \
              "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAVES" \
              "TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    MURR_LIB=$TL MURR_JIT_DEFS=$d run pmc_${n}_$i 120 rocprofv3 --pmc $ctrs --output-format csv -d $out/pmc_$n -o pass$i -- \
      "$PY" bench.py --steps 3 --warmup 1 --no-cpu --no-traffic --no-verify
  done
  "$PY" tools/pmc_sum.py $out/pmc_$n murr_jit_decode > $out/pmc_${n}_summary.txt 2>&1 || true
done
echo done
