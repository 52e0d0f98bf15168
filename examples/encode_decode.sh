#!/bin/bash
# Smoke program (the reference's src/test-seq.c + src/unit-test.sh): encode a file at k=4, n=6,
# erase the first n-k natives, decode, compare. Uses bin/RS on a GPU box, bin/CPU-RS otherwise.
set -euo pipefail
cd "$(dirname "$0")"
ROOT=..
[ -x "$ROOT/bin/RS" ] && [ -x "$ROOT/bin/CPU-RS" ] || make -C "$ROOT/csrc" -j8 >/dev/null
RS="$ROOT/bin/RS"
if ! "$ROOT/bin/RS" -h >/dev/null 2>&1 || ! python3 -c "import torch,sys; sys.exit(0 if torch.cuda.is_available() else 1)"; then
  RS="$ROOT/bin/CPU-RS"
fi
head -c 1048577 /dev/urandom > test.bin
"$RS" -k 4 -n 6 -e test.bin
"$RS" -k 4 -n 6 -e test.bin --make-conf      # conf-6-4-test.bin: keep chunks 2..5
"$RS" -d -i test.bin -c conf-6-4-test.bin -o test.out
cmp test.bin test.out && echo "round trip OK with $RS"
"$RS" -d -i test.bin -c conf -o test.identity   # examples/conf: all natives (identity decode)
cmp test.bin test.identity && echo "identity decode OK"
rm -f test.bin test.out test.identity _*_test.bin test.bin.METADATA conf-6-4-test.bin
