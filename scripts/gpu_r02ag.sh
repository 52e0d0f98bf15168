#!/bin/bash
# Round-2 session AG: wall time of the file codecs on a 1 GiB file — bin/RS streamed vs the Python
# distributed CLI (one rank) — to price the distributed CLI's Python window loop.
O=gpurun_out/r02ag
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
F=/tmp/rs_in.bin
wall() { local s=$EPOCHREALTIME; "$@"; local rc=$?; awk -v a="$s" -v b="$EPOCHREALTIME" 'BEGIN{printf "WALL_S %.3f\n", b-a}'; return $rc; }
export -f wall
step mkfile 120 python -c "import os; open('$F','wb').write(os.urandom((1<<30)+12345))" &&
step rs_stream_enc 300 bash -c "wall bin/RS -k 10 -n 14 -e $F --window 0 --no-sync -s 4" &&
step rs_inmem_enc 300 bash -c "wall bin/RS -k 10 -n 14 -e $F -s 4" &&
step dist1_enc 300 bash -c "wall python -m gpu_rscode_amd --dist -k 10 -n 14 -e $F" &&
step dist1_enc_w256 300 bash -c "wall python -m gpu_rscode_amd --dist -k 10 -n 14 -e $F --window 268435456" &&
step conf 30 bash -c "printf '/tmp/_%d_rs_in.bin\n' 4 5 6 7 8 9 10 11 12 13 > /tmp/rs_conf" &&
step dist1_dec 300 bash -c "wall python -m gpu_rscode_amd --dist -d -i $F -c /tmp/rs_conf -o /tmp/rs_out.bin && cmp $F /tmp/rs_out.bin && echo IDENTICAL" &&
step rs_stream_dec 300 bash -c "wall bin/RS -d -i $F -c /tmp/rs_conf -o /tmp/rs_out2.bin --window 0 --no-sync -s 4 && cmp $F /tmp/rs_out2.bin && echo IDENTICAL" &&
step pyimport 120 bash -c "wall python -c 'import torch, gpu_rscode_amd; torch.cuda.init()'" &&
echo SESSION-OK | tee -a $O/progress.log
