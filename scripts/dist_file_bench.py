#!/usr/bin/env python3
"""Multi-GPU file codec (``--dist``, one rank per GPU over torch.distributed) against the native
single-process windowed codec (``bin/RS --window``) on the same file.

Both run the same native window pipeline (csrc/io/stream_codec.cpp: read / GEMM / write overlapped,
pinned buffers); ``--dist`` adds torchrun, the process group, the shard bookkeeping and the CRC
combine. Each command runs ``--reps`` times, alternating, on a fresh file in ``--dir`` (page cache
warm after the first pass: the numbers compare the pipelines, not the disk). Outputs are checked
byte-identical between the two codecs and the decode against the input. Prints one JSON object.

    python scripts/dist_file_bench.py --size 1073741824 --nproc 1
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _make(path: str, size: int) -> None:
    import numpy as np

    rng = np.random.default_rng(7)
    with open(path, "wb") as f:
        left = size
        while left:
            n = min(left, 64 << 20)
            f.write(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
            left -= n


def _run(cmd: list[str], cwd: str, timeout: float) -> tuple[float, float]:
    """(process wall s, in-process codec s: bin/RS's "File codec:" line / --dist --json codec_ms)."""
    env = dict(os.environ, PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
    t0 = time.perf_counter()
    r = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True, timeout=timeout, env=env)
    dt = time.perf_counter() - t0
    if r.returncode != 0:
        raise SystemExit(f"{' '.join(cmd)} failed ({r.returncode}):\n{r.stdout[-2000:]}\n{r.stderr[-3000:]}")
    codec = None
    for line in r.stdout.splitlines():
        if line.startswith("File codec:"):
            codec = float(line.split()[2].rstrip("ms")) / 1e3
        elif line.startswith("{"):
            codec = json.loads(line)["codec_ms"] / 1e3
    if codec is None:
        raise SystemExit(f"no codec time in the output of {' '.join(cmd)}:\n{r.stdout[-2000:]}")
    return dt, codec


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--size", type=int, default=1 << 30)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--n", type=int, default=14)
    ap.add_argument("--w", type=int, default=8, choices=[8, 16])
    ap.add_argument("--window", type=int, default=0, help="bytes per chunk row per window (0: auto)")
    ap.add_argument("--nproc", type=int, default=1, help="--dist ranks (one per GPU)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--timeout", type=float, default=240)
    ap.add_argument("--staged", action="store_true", help="both codecs on the staged -s 2 pipeline (default: zero-copy)")
    a = ap.parse_args()
    base = a.dir or tempfile.mkdtemp(prefix="distbench_", dir=os.environ.get("TMPDIR", "/tmp"))
    d_rs, d_dist = os.path.join(base, "rs"), os.path.join(base, "dist")
    os.makedirs(d_rs, exist_ok=True)
    os.makedirs(d_dist, exist_ok=True)
    _make(os.path.join(d_rs, "f.bin"), a.size)
    os.link(os.path.join(d_rs, "f.bin"), os.path.join(d_dist, "f.bin"))
    rs = [os.path.join(ROOT, "bin", "RS"), "--window", str(a.window), "--no-sync"] + (["-s", "2"] if a.staged else [])
    enc = ["-k", str(a.k), "-n", str(a.n), "-w", str(a.w), "-e", "f.bin"]
    conf_names = [f"_{i}_f.bin" for i in range(a.n - a.k, a.n)]  # the reference's unit-test.sh pattern
    for d in (d_rs, d_dist):
        with open(os.path.join(d, "conf"), "w") as f:
            f.write(" ".join(conf_names) + "\n")
    dec = ["-d", "-i", "f.bin", "-c", "conf", "-o", "o.bin"]

    def dist_cmd(args):
        return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.nproc}",
                "--master-addr=127.0.0.1", f"--master-port={_port()}", "-m", "gpu_rscode_amd", "--dist", "-q",
                "--json", "--window", str(a.window), "--no-sync", *([] if a.staged else ["--zero-copy"]), *args]

    res = {f"{who}_{op}_{what}": [] for who in ("rs", "dist") for op in ("encode", "decode") for what in ("wall_s", "codec_s")}
    for _ in range(a.reps):
        for op, args in (("encode", enc), ("decode", dec)):
            for who, cmd, d in (("rs", rs + args, d_rs), ("dist", dist_cmd(args), d_dist)):
                wall, codec = _run(cmd, d, a.timeout)
                res[f"{who}_{op}_wall_s"].append(wall)
                res[f"{who}_{op}_codec_s"].append(codec)
    same = all(open(os.path.join(d_rs, f"_{i}_f.bin"), "rb").read() == open(os.path.join(d_dist, f"_{i}_f.bin"), "rb").read()
               for i in range(a.n))
    same = same and open(os.path.join(d_rs, "f.bin.METADATA")).read() == open(os.path.join(d_dist, "f.bin.METADATA")).read()

    def equal_files(x, y):
        with open(x, "rb") as fx, open(y, "rb") as fy:
            while True:
                bx, by = fx.read(1 << 24), fy.read(1 << 24)
                if bx != by:
                    return False
                if not bx:
                    return True

    decoded = all(equal_files(os.path.join(d, "o.bin"), os.path.join(d, "f.bin")) for d in (d_rs, d_dist))
    out = {"size": a.size, "k": a.k, "n": a.n, "w": a.w, "window": a.window, "nproc": a.nproc, "reps": a.reps,
           "outputs_identical": same, "decoded_ok": decoded,
           **{key: [round(v, 3) for v in vals] for key, vals in res.items()}}
    for op in ("encode", "decode"):
        for what in ("codec", "wall"):
            best_rs, best_dist = min(res[f"rs_{op}_{what}_s"]), min(res[f"dist_{op}_{what}_s"])
            out[f"{op}_{what}_GBps_rs"] = round(a.size / best_rs / 1e9, 3)
            out[f"{op}_{what}_GBps_dist"] = round(a.size / best_dist / 1e9, 3)
            out[f"{op}_{what}_dist_vs_rs"] = round(best_rs / best_dist, 3)
            # medians too: the first rep writes into fresh chunk files, later ones overwrite them
            med_rs, med_dist = statistics.median(res[f"rs_{op}_{what}_s"]), statistics.median(res[f"dist_{op}_{what}_s"])
            out[f"{op}_{what}_median_dist_vs_rs"] = round(med_rs / med_dist, 3)
    out["pipeline"] = "staged -s 2" if a.staged else "zero-copy"
    out["what"] = ("best of reps (and median ratios), page cache warm, --no-sync, GB/s = input bytes / time. codec: the file codec call "
                   "inside the process (bin/RS: encode/decode_file_stream; --dist: max over ranks from the shard "
                   "codec call to the final barrier). wall: the whole process (torchrun + interpreter + torch "
                   "import + process group for --dist)")
    print(json.dumps(out))
    return 0 if (same and decoded) else 1


if __name__ == "__main__":
    sys.exit(main())
