#!/bin/bash
# Round-2 session AE: bin/RS on a 1 GiB file with the current tree — in-memory and streamed
# (--window, bounded memory, checkpointed) encode + 4-erasure decode, byte-compared.
O=gpurun_out/r02ae
source "$(dirname "$0")/gpustep.sh"
F=/tmp/rs_in.bin
step mkfile 120 python -c "import os; open('$F','wb').write(os.urandom((1<<30)+12345))" &&
step conf 30 bash -c "printf '/tmp/_%d_rs_in.bin\n' 4 5 6 7 8 9 10 11 12 13 > /tmp/rs_conf" &&
step inmem_encode 300 bin/RS -k 10 -n 14 -e $F -s 4 &&
step inmem_decode 300 bin/RS -d -i $F -c /tmp/rs_conf -o /tmp/rs_out.bin -s 4 &&
step cmp_inmem 60 cmp $F /tmp/rs_out.bin &&
step stream_encode 300 bin/RS -k 10 -n 14 -e $F --window 0 --no-sync -s 4 &&
step stream_decode 300 bin/RS -d -i $F -c /tmp/rs_conf -o /tmp/rs_out2.bin --window 0 --no-sync -s 4 &&
step cmp_stream 60 cmp $F /tmp/rs_out2.bin &&
echo SESSION-OK | tee -a $O/progress.log
