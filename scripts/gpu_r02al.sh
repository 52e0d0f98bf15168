#!/bin/bash
# Round-2 session AL: the bench's e2e block (pinned host -> GPU -> host) at -s 4 / 32 MiB (default)
# vs -s 2 / 16 MiB and -s 4 / 16 MiB, interleaved twice.
O=gpurun_out/r02al
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
for r in a b; do
  step s4_32_$r 300 python bench.py --steps 5 --warmup 2 --streams 4 --slice 33554432 || exit 1
  step s2_16_$r 300 python bench.py --steps 5 --warmup 2 --streams 2 --slice 16777216 || exit 1
  step s4_16_$r 300 python bench.py --steps 5 --warmup 2 --streams 4 --slice 16777216 || exit 1
  step s1_16_$r 300 python bench.py --steps 5 --warmup 2 --streams 1 --slice 16777216 || exit 1
done
echo SESSION-OK | tee -a $O/progress.log
