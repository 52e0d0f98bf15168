#!/bin/bash
# One GPU-box session, parameterized:  scripts/gpu_session.sh OUTNAME RECIPE [RECIPE ...]
#
# Output goes to gpurun_out/OUTNAME/ (one log per step + progress.log). Every GPU step runs under
# its own time limit and the recipes are chained with && — after the first failure, timeout or
# fault nothing else touches the GPU (pool rules). Extra bench flags: BENCH_ARGS="...".
#
# Recipes:
#   tests      pytest -m gpu (native kernels vs the numpy oracle, RCCL world-1 paths) + smoke()
#   bench      the driver's headline command (1 GPU), plus --graph
#   presets    bench.py on every BASELINE preset (k128n160, k16n20_8g, k4n6, k16n20_64g)
#   rccl       scripts/rccl_probe.py at world 1 + bench.py --force-pg in every --comm / --scaling mode
#   files      bin/RS on a 1 GiB file: in-memory and streamed encode + 4-erasure decode, cmp
#   rcclprof   rocprofv3 kernel timelines of the one-rank RCCL group (owners/root/bcast) + no group
#   setup      bin/RS device-setup breakdown (slice sizes, serial vs overlapped)
#   prof       rocprofv3 --kernel-trace --stats of the headline and wide-stripe benches
#   pmc        PMC passes (counters only, kernel-trace) of the encode / decode / wide kernels
#   sweep      the reference's published k-sweep (scripts/sweep.py)
#   gf16       the design doc's GF(16)-method point (k=4, n=6, 1.1 GB; device + e2e)
#   lut        kbench: v_perm vs FP4 / int8 MFMA vs the LDS nibble-table kernel on every shape
#   wide       FP4 wide-stripe shapes: default kernels vs A-resident, spread vs single sink slot
#   e2efull    host pipeline sweep (streams x slice) for the full-decode and encode shapes
#   serve      small-object serving throughput: batched vs per-object launches vs hipGraph
#   decsys16   GF(2^16) decode-plan solve, host vs device (one workgroup / blocked), wide codes
#   ad hoc:    CMD="..." scripts/gpu_session.sh NAME cmd   (one step, 600 s)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
export GPURS_NO_BUILD=1
NAME=${1:?usage: gpu_session.sh OUTNAME RECIPE...}; shift
O=gpurun_out/$NAME
mkdir -p "$O"

step() {  # step NAME SECONDS CMD... : logs to $O/NAME.log, one progress line before and after
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a "$O/progress.log"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a "$O/progress.log"
  [ $rc -ne 0 ] && tail -20 "$O/$name.log"
  return $rc
}
PY="python3 -u"
PROF="rocprofv3 --kernel-trace --stats --output-format csv -o run"

r_tests() {
  step pytest_gpu 1000 $PY -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread &&
  step smoke 300 $PY -c "import __graft_entry__ as g; g.smoke()"
}
r_bench() {
  step bench 300 $PY bench.py --gpus 1 --steps 20 --warmup 5 $BENCH_ARGS &&
  step bench_graph 300 $PY bench.py --graph --no-e2e $BENCH_ARGS
}
r_presets() {
  step bench_k128n160 300 $PY bench.py --preset k128n160 --steps 20 &&
  step bench_k16n20_8g 300 $PY bench.py --preset k16n20_8g --steps 10 &&
  step bench_k4n6 300 $PY bench.py --preset k4n6 &&
  step bench_k16n20_64g 600 $PY bench.py --preset k16n20_64g --steps 5 --warmup 1
}
r_rccl() {
  step rccl_probe 180 $PY scripts/rccl_probe.py &&
  step bench_pg_headline 300 $PY bench.py --force-pg --steps 10 --warmup 2 --no-e2e &&
  step bench_pg_strong 300 $PY bench.py --force-pg --scaling strong --steps 10 --warmup 2 --no-e2e
}
r_files() {
  local F=/tmp/rs_in.bin
  step mkfile 120 $PY -c "import os; open('$F','wb').write(os.urandom((1<<30)+12345))" &&
  step conf 30 bash -c "printf '/tmp/_%d_rs_in.bin\n' 4 5 6 7 8 9 10 11 12 13 > /tmp/rs_conf" &&
  step inmem_encode 300 bin/RS -k 10 -n 14 -e $F -s 2 &&
  step inmem_decode 300 bin/RS -d -i $F -c /tmp/rs_conf -o /tmp/rs_out.bin -s 2 &&
  step cmp_inmem 60 cmp $F /tmp/rs_out.bin &&
  step stream_encode 300 bin/RS -k 10 -n 14 -e $F --window 0 --no-sync -s 4 &&
  step stream_decode 300 bin/RS -d -i $F -c /tmp/rs_conf -o /tmp/rs_out2.bin --window 0 --no-sync -s 4 &&
  step cmp_stream 60 cmp $F /tmp/rs_out2.bin
}
r_setup() {  # bin/RS device + host setup breakdown, 1 GiB encode + decode (THP-pinned vs hipHostMalloc)
  local F=/tmp/rs_in.bin
  step mkfile2 120 $PY -c "import os; open('$F','wb').write(os.urandom((1<<30)+12345))" &&
  step conf2 30 bash -c "printf '/tmp/_%d_rs_in.bin\\n' 4 5 6 7 8 9 10 11 12 13 > /tmp/rs_conf" &&
  step setup_enc 120 bin/RS -k 10 -n 14 -e $F -s 2 &&
  step setup_dec 120 bin/RS -d -i $F -c /tmp/rs_conf -o /tmp/rs_out.bin -s 2 &&
  step setup_cmp 60 cmp $F /tmp/rs_out.bin &&
  step setup_enc2 120 bin/RS -k 10 -n 14 -e $F -s 2 &&
  step setup_dec2 120 bin/RS -d -i $F -c /tmp/rs_conf -o /tmp/rs_out.bin -s 2 &&
  step setup_enc_hhm 120 env GFRS_HOST_ALLOC=hipHostMalloc bin/RS -k 10 -n 14 -e $F -s 2 &&
  step setup_dec_hhm 120 env GFRS_HOST_ALLOC=hipHostMalloc bin/RS -d -i $F -c /tmp/rs_conf -o /tmp/rs_out.bin -s 2 &&
  step setup_enc_serial 120 env GFRS_TUNE=setup=serial bin/RS -k 10 -n 14 -e $F -s 2 &&
  step setup_stream_enc 120 bin/RS -k 10 -n 14 -e $F --window 0 --no-sync -s 4 &&
  step setup_stream_dec 120 bin/RS -d -i $F -c /tmp/rs_conf -o /tmp/rs_out2.bin --window 0 --no-sync -s 4 &&
  step setup_cmp2 60 cmp $F /tmp/rs_out2.bin
}
r_prof() {
  step prof_k10 300 $PROF -d $O/prof_k10 -- python3 bench.py --steps 20 --no-e2e &&
  step prof_k128 300 $PROF -d $O/prof_k128 -- python3 bench.py --preset k128n160 --steps 20 --no-e2e &&
  step prof_k16 300 $PROF -d $O/prof_k16 -- python3 bench.py --preset k16n20_8g --steps 10 --no-e2e
}
r_decsys16() {  # GF(2^16) decode-plan solve: host vs device (one workgroup / blocked)
  step decsys16 300 $PY scripts/decsys16_bench.py
}
r_rcclprof() {  # kernel timelines: RCCL kernels on their own stream beside the GEMMs (one-rank group)
  local m
  for m in owners root bcast; do
    step trace_pg_$m 300 rocprofv3 --kernel-trace --output-format csv -o run -d $O/trace_pg_$m -- \
      python3 bench.py --force-pg --comm $m --no-compare --no-e2e --steps 20 --warmup 3 &&
    $PY scripts/trace_overlap.py $O/trace_pg_$m --last 60 --out $O/timeline_pg_$m.txt > /dev/null || return 1
  done
  step trace_nopg 300 rocprofv3 --kernel-trace --output-format csv -o run -d $O/trace_nopg -- \
    python3 bench.py --no-e2e --steps 20 --warmup 3 &&
  $PY scripts/trace_overlap.py $O/trace_nopg --last 60 --out $O/timeline_nopg.txt > /dev/null
}
r_pmc() {
  local C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
  local C2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
  local C3="FETCH_SIZE"
  local C4="WRITE_SIZE"
  local cfg name args i ctr
  local cases=("enc10:--k 10 --m 4" "dec10:--k 10 --m 4 --copies 6" "wide_mfma:--k 128 --m 32 --engine mfma")
  [ -n "$PMC_CASES" ] && IFS=';' read -ra cases <<< "$PMC_CASES"  # "name:args;name:args"
  for cfg in "${cases[@]}"; do
    name=${cfg%%:*}; args=${cfg#*:}; i=0
    for ctr in "$C1" "$C2" "$C3" "$C4"; do
      i=$((i+1))
      step pmc_${name}_$i 120 rocprofv3 --kernel-trace --pmc $ctr -d $O/pmc_${name}_$i -o run --output-format csv -- \
        python3 scripts/prof_case.py --iters 3 $args || return 1
    done
  done
}
r_sweep() { step sweep 1200 $PY scripts/sweep.py --part gpu --out $O/sweep_gpu.json; }
r_gf16() { step gf16 300 $PY scripts/sweep.py --part gf16 --out $O/gf16.json; }
r_lut() {  # LDS nibble-table ablation next to v_perm and the matrix-core kernels (kbench, interleaved rounds)
  step kbench_lut 600 $PY scripts/kbench.py --rounds 3 --reps 5 --variants "None;mfma;mfma_i8;lut" --out $O/kbench_lut.json
}
r_wide() {  # wide-stripe FP4 kernel shapes (k=128, m rebuilt rows, with / without fused copies): A/B of kernel choices
  local i
  for i in 1 2; do
    step wide_default_$i 300 $PY scripts/fp4_shapes.py ${WIDE_MS:-20,24,26,28,32} &&
    step wide_v1_$i 300 env GFRS_TUNE=fp4=v1 $PY scripts/fp4_shapes.py ${WIDE_MS:-20,24,26,28,32} &&
    step wide_ar_$i 300 env GFRS_TUNE=fp4=ar $PY scripts/fp4_shapes.py ${WIDE_MS:-20,24,26,28,32} &&
    step wide_tm_$i 300 env GFRS_TUNE=fp4=tm $PY scripts/fp4_shapes.py ${WIDE_MS:-20,24,26,28,32} || return 1
  done
}
r_e2efull() {  # host pipeline, the reference's decode shape (k=10 in, all 10 natives out) and the encode shape
  step pipe_full 300 $PY scripts/pipe_bench.py --m 10 --streams 1,2,3,4 --split 1 --rect 1 \
    --slices 8388608,16777216,33554432 &&
  step pipe_enc 300 $PY scripts/pipe_bench.py --m 4 --streams 1,2,3,4 --split 1 --rect 1 --slices 8388608,16777216,33554432
}
r_serve() { step serve 600 $PY scripts/serve_bench.py --out $O/serve.json; }
r_cmd() { step cmd 600 bash -c "$CMD"; }

rc=0
for r in "$@"; do
  "r_$r" || { rc=$?; echo "[$(date +%T)] recipe $r FAILED rc=$rc" | tee -a "$O/progress.log"; break; }
done
[ $rc -eq 0 ] && echo "SESSION-OK $*" | tee -a "$O/progress.log"
exit $rc
