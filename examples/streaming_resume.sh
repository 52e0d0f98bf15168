#!/bin/bash
# Bounded-memory streaming codec with checkpoint/resume: encode a file in column
# windows, "crash" part-way (the test hook stop_after, via the Python binding), resume with the CLI,
# then decode with 4 erasures in windows and compare. Uses bin/RS on a GPU box, bin/CPU-RS otherwise.
set -euo pipefail
cd "$(dirname "$0")"
ROOT=..
[ -x "$ROOT/bin/RS" ] && [ -x "$ROOT/bin/CPU-RS" ] || make -C "$ROOT/csrc" -j8 >/dev/null
RS="$ROOT/bin/RS"
if ! python3 -c "import torch,sys; sys.exit(0 if torch.cuda.is_available() else 1)"; then RS="$ROOT/bin/CPU-RS"; fi
head -c 50000017 /dev/urandom > big.bin
# simulated crash after 3 windows of 1 MiB per chunk (leaves big.bin.PROGRESS, no METADATA)
PYTHONPATH="$ROOT" python3 -c "
from gpu_rscode_amd._native import cpu
r = cpu().encode_file_stream('big.bin', 10, 4, window=1 << 20, stop_after=3, durable=False)
print('interrupted after', r['windows'], 'windows; complete =', r['complete'])"
cat big.bin.PROGRESS | cut -c1-80; echo ...
"$RS" -k 10 -n 14 -e big.bin --window 2097152   # resumes at the checkpoint (any window size)
printf '_%d_big.bin\n' 0 2 3 5 6 8 10 11 12 13 > conf-big
"$RS" -d -i big.bin -c conf-big -o big.out --window 0
cmp big.bin big.out && echo "streamed round trip OK with $RS"
rm -f big.bin big.out _*_big.bin big.bin.METADATA conf-big
