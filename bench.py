#!/usr/bin/env python3
"""Headline benchmark: Reed-Solomon encode + decode throughput at k=10, n=14 on 1 GiB per GPU.

Metric (BASELINE.json): "encode+decode throughput (GB/s) at k=10,n=14 on 1 GiB; 1/2/4/8-GPU scaling".

``python bench.py --gpus N`` runs N ranks, one process per GPU over RCCL. When WORLD_SIZE is not
set (a plain ``python bench.py --gpus 8``) the process re-launches itself through
``torch.distributed.run`` as a CHILD before touching any GPU and exits with the child's status;
under torchrun (the driver's launch) every rank checks WORLD_SIZE == --gpus.

One step on every rank:
  1. encode:  parity[4, C] = E . data[10, C]                          (gfx950 v_perm GF-GEMM)
  2. decode:  4 random erased chunks (natives AND parity, at least one native) drawn from a pool
              of recoverable patterns. The pattern lives in device memory: rank 0 takes it from the
              device-resident pool and RCCL-broadcasts it to every rank (a lost node takes the same
              chunk index from every stripe — the reference's one shared decode system,
              src/decode.cu:375). Each rank then checks it, solves the systematic
              e x (e+k) decode system and writes the decode plan (row pointers + tables) ON DEVICE
              (ops.PatternDecoder; on a side stream, one step ahead), and one fused pass rebuilds the
              erased natives and copies the surviving ones into a fresh [10, C] output. The
              broadcast itself runs --bcast-ahead (2) steps ahead on a stream of its own, into a
              ring of pattern slots, so a late RCCL kernel never delays a solve.
Consecutive steps alternate between two lanes (--lanes 2: a stream, a parity slot, a decode output
and a decode plan each), so step i+1's encode runs into the launch gap and the tail wave of step
i's decode (every step still encodes and decodes its whole stripe).
C = ceil(2^30 / 10) = 107374183 bytes (odd, as in the reference, src/encode.cu:317). Data is synthetic
random bytes generated in HBM; E and the pattern pool are RCCL-broadcast from rank 0 at setup.

Headline (N > 1): weak scaling, --comm bcast. Every GPU encodes and decodes its own 1 GiB stripe and
keeps its parity and decoded rows in its own HBM — exactly what the N = 1 number does — and the
step's RCCL traffic is the pattern broadcast. The same record also carries, each timed in its own
barrier-bracketed loop:
  value_by_comm   per-step parity movement on top of the headline step:
                    owners — one all_to_all placing parity chunk-contiguously (1/N of every block
                             over every xGMI link); root — every peer's whole parity block into rank 0
                             (the reference's gather, src/encode.cu:410-429, as grouped send/recv);
                    none   — no per-step traffic at all (each rank draws the pattern itself)
  value_strong    the reference's multi-GPU semantics: ONE 1 GiB stripe column-sharded over the N
                  ranks (src/encode.cu:368-381), every step ending with the gather of parity and
                  decoded natives into rank 0's full rows (in place, one link per peer)
  value_no_comm   = value_by_comm.none
Moving 0.43 GB of parity per step over xGMI costs more than the 0.65 ms step itself (~64 GB/s per
link direction against ~5 TB/s of HBM), so those numbers measure the links; the headline measures
the codec the way N = 1 does. --comm / --scaling choose the headline explicitly.

value = (encoded bytes + decoded bytes) over all ranks / max-over-ranks step time, in GB/s (1e9).

Failure isolation (N > 1). The headline is timed, verified and reduced FIRST (step_ms_by_rank shows
every rank's own step time, so a straggler is visible). Only then do the comparison modes run, one
at a time (e2e, none, owners, strong, root: least collective risk first), each in its own try under
one watchdog (--compare-budget). A mode that raises is recorded as {"error": ...} and no further
collective is issued (the group may be out of step); a mode that hangs (an RCCL peer that never
joins) is cut off by the watchdog, which prints the record held so far. Either way rank 0 prints the
ONE JSON line with the verified headline. init_process_group gets a bounded timeout (--pg-timeout,
longer than both budgets). Fault injection: GFRS_FAULT_MODE=owners|root|strong [GFRS_FAULT_RANK=r]
[GFRS_FAULT_KIND=hang] (gpu_rscode_amd/parallel/placement.py: maybe_fault).

--force-pg (or GFRS_FORCE_PG=1) creates a one-rank RCCL process group at N = 1: the broadcast, the
all_to_all, the grouped send/recv and the strong-scaling gather then run against rank 0 itself, so
every RCCL code path of the N > 1 run executes on a single MI355X. --pg-backend gloo rehearses N
ranks on one GPU (every mode; point-to-point pieces staged through host memory).

Reference comparison. The reference's published MB/s is PCIe-inclusive: H2D + kernel + D2H
(src/encode.cu:117-119,228-232, src/decode.cu:96-98,186-190, doc/design.tex:482-500). Its nearest
published point to k=10, n=14 is k=8, n=11 on 1.1 GB (Tesla C2050): encode 695.00 ms + decode
1026.68 ms (doc/result-graph/Total-GPU-{en,de}coding-time-3.pdf) = 2 * 1,096,310,784 B / 1.72168 s =
1.2736 GB/s. Two ratios are reported, labelled:
  vs_baseline      the like-for-like one (= e2e.vs_baseline_e2e; null when the e2e timing did not run):
                   pinned host -> H2D -> kernel -> D2H encode and decode
                   of the same 1 GiB stripe (-s 2 streams, every rank concurrently on its own PCIe
                   link), survivors read from host memory, erased natives rebuilt to host memory;
                   e2e.decode_full_GBps is the reference's exact decode shape (the whole k x k
                   inverse applied, all k natives D2H into one contiguous file image);
  vs_baseline_device  device-resident value / 1.2736 (not like for like: the reference's number
                   includes PCIe both ways).
"""
from __future__ import annotations

import os

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this driver (RCCL peers)

import argparse  # noqa: E402
import datetime  # noqa: E402
import json  # noqa: E402
import socket  # noqa: E402
import subprocess  # noqa: E402
import sys  # noqa: E402
import threading  # noqa: E402
import time  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from gpu_rscode_amd import gf  # noqa: E402
from gpu_rscode_amd.models import ReedSolomon, alloc_rows, flat_rows  # noqa: E402
from gpu_rscode_amd.parallel.dist import shard_range  # noqa: E402
from gpu_rscode_amd.parallel.placement import ParityExchange, StripeGather  # noqa: E402
from gpu_rscode_amd.utils.timing import trace_range  # noqa: E402

BASELINE_GBPS = 2 * 1_096_310_784 / 1.72168 / 1e9  # 1.2736 GB/s
METRIC = "encode+decode throughput (GB/s) at k=10,n=14 on 1 GiB; 1/2/4/8-GPU scaling"
COMM_MODES = ("bcast", "owners", "root", "none")
# BASELINE.json's other configs (#4, #5, #1's shape at GPU scale) and the w = 16 field, timed by the
# headline run itself (N = 1) so the driver's record carries them
CONFIG_PRESETS = ("k128n160", "k16n20_8g", "k4n6", "k10n14_w16", "k4n6_cpu")

# BASELINE.json configs. Weak presets are per GPU; strong presets are the whole job's bytes.
PRESETS = {
    "k10n14": dict(k=10, n=14, bytes=1 << 30, erasures=4),
    # (two lanes, the default: with alloc_rows' skewed 640 MiB pitch 4.72-4.77 ms/step against
    # 4.94-4.96 with one lane; at the old 512 MiB pitch one lane had won, 5.00 vs 5.06-5.10:
    # profiles/headline/r09_k16)
    "k16n20_8g": dict(k=16, n=20, bytes=8 << 30, erasures=4),
    # config #4 as one stripe: 64 GiB column-sharded over the ranks (8 GiB each at N = 8), parity and
    # decoded natives gathered into rank 0 once after the timed loop (timed on its own)
    "k16n20_64g": dict(k=16, n=20, bytes=64 << 30, erasures=4, scaling="strong", gather="end", lanes=1),
    "k128n160": dict(k=128, n=160, bytes=1 << 30, erasures=32),
    "k4n6": dict(k=4, n=6, bytes=1_096_310_784, erasures=2),
    # the reference's w = 16 field (src/galoisfield.cu:22-32), same stripe shape as the headline
    "k10n14_w16": dict(k=10, n=14, bytes=1 << 30, erasures=4, field="gf65536"),
    # BASELINE config #1: k=4, n=6 on the CPU, 1 MiB (the C++ CPU codec; src/cpu-rs.c's shape)
    "k4n6_cpu": dict(k=4, n=6, bytes=1 << 20, erasures=2, device="cpu"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=None, help="ranks / GPUs (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--min-warmup-ms", type=float, default=None,
                    help="before the --warmup steps, run local steps (no collectives) until this many ms have "
                         "passed, so the timed steps start at sustained clocks (default 250 on cuda, 0 on cpu; "
                         "GFRS_MIN_WARMUP_MS; 0: off)")
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--bytes", type=int, default=None, help="input bytes per GPU (weak) / in total (strong)")
    ap.add_argument("--erasures", type=int, default=None)
    ap.add_argument("--field", default=None, choices=["gf256", "gf65536"],
                    help="symbol field: GF(2^8) (default) or GF(2^16) (16-bit symbols, poly 0x1100B)")
    ap.add_argument("--comm", default="bcast", choices=COMM_MODES, help="per-step RCCL traffic (headline mode)")
    ap.add_argument("--scaling", default=None, choices=["weak", "strong"],
                    help="weak: a stripe per GPU (default); strong: one stripe column-sharded over all GPUs")
    ap.add_argument("--gather", default=None, choices=["step", "end", "none"],
                    help="strong scaling: gather parity + decoded natives into rank 0 every step (default), "
                         "once after the timed loop, or never")
    ap.add_argument("--force-pg", action="store_true",
                    help="N = 1: create a one-rank RCCL process group and run every collective against itself")
    ap.add_argument("--no-compare", action="store_true", help="skip timing the other --comm / --scaling modes")
    ap.add_argument("--no-e2e", action="store_true", help="skip the pinned host->device->host timing")
    ap.add_argument("--e2e", action="store_true", help=argparse.SUPPRESS)  # (on by default)
    # e2e -s 2 / 16 MiB: profiles/host_pipeline/r02al (52.0 GB/s against 51.2 at -s 4 / 32 MiB)
    ap.add_argument("--streams", type=int, default=2, help="e2e: HIP streams (-s) per GPU")
    ap.add_argument("--slice", type=int, default=16 << 20, help="e2e: column slice per stream step")
    ap.add_argument("--vec", type=int, default=None, help="kernel variant: 16-byte groups per lane (ablation)")
    ap.add_argument("--pf", type=int, default=2, help="kernel variant: rows in flight (with --vec)")
    ap.add_argument("--nt", action="store_true", help="kernel variant: non-temporal (with --vec)")
    ap.add_argument("--no-overlap", action="store_true", help="solve on the main stream (no side stream)")
    ap.add_argument("--side-priority", action="store_true",
                    help="create the side stream (decode-system solve) with high priority")
    ap.add_argument("--bcast-ahead", type=int, default=2,
                    help="bcast: steps a pattern's broadcast runs ahead of the step that solves it (0: in line)")
    ap.add_argument("--lanes", type=int, default=None,
                    help="streams that consecutive steps alternate between (own parity slot + decode output)")
    ap.add_argument("--preset", default="k10n14", choices=sorted(PRESETS),
                    help="BASELINE.json config: k10n14 (headline, #2/#3), k16n20_8g (#4 per GPU), k16n20_64g "
                         "(#4 as one 64 GiB stripe), k128n160 (#5), k4n6 (the reference's published shape)")
    ap.add_argument("--engine", default="auto", choices=["auto", "valu", "mfma"],
                    help="encode GEMM engine, GF(2^8) and GF(2^16) (auto: FP4 matrix cores for wide stripes, v_perm otherwise)")
    ap.add_argument("--graph", action="store_true", help="replay each step from a captured hipGraph (N = 1)")
    ap.add_argument("--pg-backend", default=None, choices=["nccl", "gloo"],
                    help="process-group backend (default: nccl = RCCL on cuda, gloo on cpu). gloo on cuda "
                         "rehearses N ranks on fewer GPUs: ranks wrap round the visible devices (RCCL refuses two "
                         "ranks on one GPU); point-to-point pieces are staged through host memory")
    ap.add_argument("--headline-budget", type=float, default=float(os.environ.get("GFRS_HEADLINE_BUDGET_S", 600)),
                    help="seconds for setup + the headline loop + its verification; past it rank 0 prints an "
                         "error record and every rank exits")
    ap.add_argument("--compare-budget", type=float, default=float(os.environ.get("GFRS_COMPARE_BUDGET_S", 180)),
                    help="seconds for all comparison modes (value_by_comm, strong, e2e) after the headline; a "
                         "mode still running then is recorded as timed out and the headline record printed")
    ap.add_argument("--pg-timeout", type=float, default=float(os.environ.get("GFRS_PG_TIMEOUT_S", 900)),
                    help="process-group timeout (init_process_group(timeout=)); longer than both budgets")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: the C++ CPU codec over gloo (launcher / communication plumbing on a host)")
    ap.add_argument("--configs", default=None,
                    help="N = 1: after the headline, time these presets (comma list) each in a fresh child "
                         "process and embed their records under configs (default on cuda with the k10n14 "
                         f"headline: {','.join(CONFIG_PRESETS)}; 'none': off)")
    ap.add_argument("--config-steps", type=int, default=20, help="timed steps of each --configs child")
    ap.add_argument("--config-warmup", type=int, default=5, help="warmup steps of each --configs child")
    ap.add_argument("--configs-budget", type=float, default=float(os.environ.get("GFRS_CONFIGS_BUDGET_S", 150)),
                    help="seconds for all --configs children together (each gets what is left, at most 75)")
    a = ap.parse_args(argv)
    pr = {"scaling": "weak", "gather": "step", "lanes": 2, "field": "gf256", **PRESETS[a.preset]}
    pr.pop("device", None)  # (selects the config child's --device; the command line decides here)
    for key, val in pr.items():
        if getattr(a, key) is None:
            setattr(a, key, val)
    if a.device == "cpu" and "--bytes" not in " ".join(argv if argv is not None else sys.argv):
        a.bytes = 1 << 20  # plumbing runs: 1 MiB per rank
    if a.configs is None:
        headline = a.preset == "k10n14" and a.bytes == PRESETS["k10n14"]["bytes"] and a.field == "gf256"
        a.configs = ",".join(CONFIG_PRESETS) if (a.device == "cuda" and headline and not a.graph) else "none"
    a.configs = [] if a.configs in ("", "none") else [c for c in a.configs.split(",") if c]
    bad = [c for c in a.configs if c not in PRESETS]
    if bad:
        ap.error(f"--configs: unknown preset(s) {bad}")
    if a.min_warmup_ms is None:
        a.min_warmup_ms = float(os.environ.get("GFRS_MIN_WARMUP_MS", 250 if a.device == "cuda" else 0))
    a.force_pg = a.force_pg or os.environ.get("GFRS_FORCE_PG") == "1"
    if a.pg_backend is None:
        a.pg_backend = "nccl" if a.device == "cuda" else "gloo"
    if a.device == "cpu" and a.pg_backend != "gloo":
        ap.error("--device cpu runs over gloo")
    a.rehearsal = a.device == "cuda" and a.pg_backend == "gloo"
    if a.rehearsal and a.graph:
        ap.error("--pg-backend gloo on cuda: no --graph (a rehearsal has per-step host staging)")
    return a


# ---- launcher --------------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(gpus: int, argv: list[str]) -> int:
    """Run this script under torch.distributed.run with ``gpus`` ranks as a child process (this
    process has not touched a GPU and never execs) and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    return subprocess.run(cmd, env=dict(os.environ)).returncode


# ---- workloads -------------------------------------------------------------------------------
def erasure_pool(k: int, n: int, erasures: int, rs: ReedSolomon, size: int = 16) -> list[list[int]]:
    """Recoverable survivor lists with `erasures` random chunks of the n lost (natives and parity
    alike), at least one native among them — BASELINE config #3's "4 random erasures". Patterns
    with the same number of erased natives share one device-built decode plan."""
    rng = np.random.default_rng(1234)
    pool = []
    while len(pool) < size:
        erased = set(rng.choice(n, size=erasures, replace=False).tolist())
        rows = [r for r in range(n) if r not in erased]
        if any(e < k for e in erased) and rs.is_recoverable(rows):
            pool.append(rows)
    return pool


def _check_windows(C: int, width: int = 1 << 16, even: bool = False) -> list[tuple[int, int]]:
    """Head, middle and ragged-tail column windows used to check full parity rows (``even``: whole
    16-bit symbols, C even)."""
    mid = C // 2 - width // 2
    if even:
        mid -= mid % 2
    wins = {(0, min(C, width)), (max(0, mid), min(C, mid + width)), (max(0, C - width), C)}
    return sorted(wins)


def _oracle_gemm(e_mat: np.ndarray, x: np.ndarray, wide: bool) -> np.ndarray:
    """numpy GF oracle of parity = E . x over byte rows (GF(2^16): little-endian 16-bit symbols)."""
    if not wide:
        return gf.GF256.gemm(e_mat, x)
    out = gf.field(16).gemm(e_mat, np.ascontiguousarray(x).view("<u2"))
    return np.ascontiguousarray(out.astype("<u2")).view(np.uint8)


class GpuWorkload:
    """Encode + device-built decode plan + fused decode on one MI355X (the HIP kernels)."""

    def __init__(self, a, k, n, C, e_mat, g, pool_dev, rank, dev, slots, parity_bufs=None, out_bufs=None, seed=None):
        from gpu_rscode_amd._native import hip
        from gpu_rscode_amd.ops import GemmPlan, PatternDecoder, fill_random_

        hip()  # fail loudly if the native extension is missing
        self.a, self.k, self.p, self.C, self.rank = a, k, n - k, C, rank
        self.wide = a.field == "gf65536"
        self.lanes = 1 if a.graph else max(1, a.lanes)
        slots = max(slots, self.lanes)
        self.data = alloc_rows(k, C, dev)
        fill_random_(flat_rows(self.data),
                     seed=rank + 1 if seed is None else seed)
        self.parity = parity_bufs or [alloc_rows(self.p, C, dev) for _ in range(slots)]
        self.outs = out_bufs or [alloc_rows(k, C, dev) for _ in range(self.lanes)]
        if self.wide:  # GF(2^16): the generator as 16-bit words, the v_perm w = 16 engine
            from gpu_rscode_amd.ops import Gemm16Plan
            self.g_dev = torch.from_numpy(np.ascontiguousarray(g, dtype="<u2").view(np.int16)).to(dev)
        else:
            self.g_dev = torch.from_numpy(np.ascontiguousarray(g)).to(dev)
        self.e_mat = e_mat
        self.pool_dev = pool_dev
        # erased natives per pool pattern (known on the host: it picks the plan shape, the pattern
        # itself only ever travels on the device)
        self.e_of = [k - sum(1 for r in rows if r < k) for rows in pool_dev.tolist()]
        self.enc = [Gemm16Plan(self.data, par, e_mat, engine=a.engine) if self.wide
                    else GemmPlan(self.data, par, e_mat, engine=a.engine) for par in self.parity]
        # one device-built decode plan per (slot, number of erased natives)
        self.dec = [{e: PatternDecoder(self.g_dev, [self.data[i] for i in range(k)] + [par[i] for i in range(self.p)],
                                       [self.outs[s % self.lanes][i] for i in range(k)], e)
                     for e in sorted(set(self.e_of))}
                    for s, par in enumerate(self.parity)]
        self.streams = [torch.cuda.Stream(dev) for _ in range(self.lanes)]  # non-default (hipGraph capture)
        self.stream = self.streams[0]
        torch.cuda.set_stream(self.stream)
        # pattern + decode-system solve overlap the encode GEMM
        self.side = torch.cuda.Stream(dev, priority=-1) if a.side_priority else torch.cuda.Stream(dev)
        self.inv_done = torch.cuda.Event()
        self.kv = {} if self.wide else dict(vec=a.vec, pf=a.pf, nt=a.nt)
        self.graph_mode = False
        self.bcast = False  # rank 0 RCCL-broadcasts each step's pattern (set per timed mode)
        # Look-ahead broadcast: step j's pattern is broadcast on its own stream while step j - ahead
        # is issued, into ring slot j % R; the solve of step j waits for that one broadcast only. An
        # RCCL kernel can sit queued behind a GEMM's workgroups for hundreds of microseconds (a small
        # copy kernel on another queue waited 150-600 us in profiles/multigpu/r03_rccl), and its peers hold
        # theirs until it starts, so in-line broadcasting would put that wait on the solve's path.
        self.ahead = max(0, a.bcast_ahead)
        self.ring = torch.empty((self.ahead + 2, k), dtype=torch.int32, device=dev)
        self.pat_stream = torch.cuda.Stream(dev)
        self.pat_ready = [torch.cuda.Event() for _ in range(self.ahead + 2)]
        self.pat_free = [torch.cuda.Event() for _ in range(self.ahead + 2)]
        self.bcast_next = None

    def flat_parity(self, slot: int) -> torch.Tensor:
        par = self.parity[slot]
        return flat_rows(par)

    def piece_rows(self, slot: int) -> list[torch.Tensor]:
        """The rows a strong-scaling gather moves for `slot`: parity, then the decoded natives."""
        return [self.parity[slot][i] for i in range(self.p)] + [self.outs[slot % self.lanes][i] for i in range(self.k)]

    def lane_stream(self, slot: int):
        """The stream of the lane that owns parity slot `slot`."""
        return self.streams[slot % self.lanes]

    def use_lane(self, slot: int) -> None:
        """Make slot's lane stream current: the step's kernels and the exchange of its parity (and
        the wait before that parity buffer is overwritten) are ordered on it."""
        self.stream = self.lane_stream(slot)
        torch.cuda.set_stream(self.stream)

    def _prepare(self, i: int, dec, stream) -> None:
        """Step i's pattern (rank 0 takes it from the device-resident pool; with bcast every other
        rank receives it over RCCL into its decoder's rows), then the on-device check + solve + plan
        build — all ordered on `stream`, no copies."""
        with torch.cuda.stream(stream):
            src = self.pool_dev[i % self.pool_dev.shape[0]] if (self.rank == 0 or not self.bcast) else dec.rows
            if self.bcast:
                dist.broadcast(src, 0)
            dec.solve(stream, rows=src)
        dec.last_i = i

    def step(self, i: int, slot: int) -> None:
        """One encode + one device-built decode plan + one decode GEMM.

        Default schedule: the plan of step i+1 is built on a side stream right after step i's decode
        GEMM is queued, so the one-workgroup solve runs beside that GEMM. Each lane's decoder waits
        for the previous decode that read its descriptor (event per decoder)."""
        dec = self._dec(i, slot)
        if self.a.no_overlap:  # everything on one stream, plan first
            self._prepare(i, dec, self.stream)
            self.enc[slot].run(**self.kv)
            dec.run(**self.kv)
            return
        if self.graph_mode:  # captured per pattern: plan built under this step's encode
            self.side.wait_stream(self.stream)
            self._prepare(i, dec, self.side)
            self.inv_done.record(self.side)
            self.enc[slot].run(**self.kv)
            self.stream.wait_event(self.inv_done)
            dec.run(**self.kv)
            return
        if not getattr(dec, "pending", False):  # (first step of a loop)
            self._issue(i, dec)
        self.enc[slot].run(**self.kv)
        self.stream.wait_event(dec.solved)
        dec.run(**self.kv)
        dec.used.record(self.stream)
        dec.pending = False
        nxt_slot = (i + 1) % len(self.dec)
        self._issue(i + 1, self._dec(i + 1, nxt_slot), self.lane_stream(nxt_slot))

    def _dec(self, i: int, slot: int):
        return self.dec[slot][self.e_of[i % len(self.e_of)]]

    def reset(self) -> None:
        """Start a loop with no plan in flight: its first step builds its own (so a timed loop of K
        steps builds K + 1 plans — one more than it needs)."""
        for decs in self.dec:
            for dec in decs.values():
                dec.pending = False
        self.bcast_next = None  # every rank restarts the broadcast sequence at the loop's first step

    def _bcast_until(self, j: int) -> None:
        """Issue the pattern broadcasts of every step up to j (same sequence on every rank)."""
        R, P = len(self.ring), self.pool_dev.shape[0]
        while self.bcast_next <= j:
            t, s = self.bcast_next, self.bcast_next % R
            with torch.cuda.stream(self.pat_stream):
                # every rank, rank 0 included, solves from the ring (one code path: a one-rank RCCL
                # group on one GPU runs the same slots and events as the peers of an 8-GPU job)
                self.pat_stream.wait_event(self.pat_free[s])  # the solve that last read slot s
                if self.rank == 0:
                    self.ring[s].copy_(self.pool_dev[t % P])
                dist.broadcast(self.ring[s], 0)
                self.pat_ready[s].record(self.pat_stream)
            self.bcast_next += 1

    def _issue(self, i: int, dec, stream=None) -> None:
        if not hasattr(dec, "solved"):
            dec.solved, dec.used = torch.cuda.Event(), torch.cuda.Event()
            dec.used.record(stream or self.stream)
        self.side.wait_event(dec.used)  # the last decode that read this descriptor is done
        if self.bcast and self.ahead > 0:
            if self.bcast_next is None:
                self.bcast_next = i
            self._bcast_until(i + self.ahead)
            s = i % len(self.ring)
            self.side.wait_event(self.pat_ready[s])
            with torch.cuda.stream(self.side):
                dec.solve(self.side, rows=self.ring[s])
            self.pat_free[s].record(self.side)
            dec.last_i = i
        else:
            self._prepare(i, dec, self.side)
        dec.solved.record(self.side)
        dec.pending = True

    def sync(self) -> None:
        torch.cuda.synchronize()

    def verify(self) -> bool:
        """Every decoder's last pattern solved (status 0), every decoded output equals the data in
        full, and every parity slot matches the numpy oracle at its head, middle and ragged tail."""
        ok = all(int(d.status.item()) == 0 for decs in self.dec for d in decs.values())
        # each decoder's last plan was built for the pattern of the step it was issued for (on a
        # rank other than 0 that pattern only ever arrived by the step's broadcast)
        pool = self.pool_dev.tolist()
        for decs in self.dec:
            for d in decs.values():
                if hasattr(d, "last_i"):
                    want = sorted(set(range(self.k)) - set(pool[d.last_i % len(pool)]))
                    ok = ok and sorted(d.erased.tolist()) == want
        ok = ok and all(torch.equal(out, self.data) for out in self.outs)
        for a, b in _check_windows(self.C, even=self.wide):
            want = _oracle_gemm(self.e_mat, self.data[:, a:b].cpu().numpy(), self.wide)
            ok = ok and all(np.array_equal(par[:, a:b].cpu().numpy(), want) for par in self.parity)
        return bool(ok)


class CpuWorkload:
    """The same step on host tensors through the C++ CPU codec (gloo plumbing runs)."""

    def __init__(self, a, k, n, C, e_mat, g, pool_dev, rank, slots, parity_bufs=None, out_bufs=None, seed=None):
        self.k, self.p, self.C, self.rank = k, n - k, C, rank
        self.wide = a.field == "gf65536"
        self.rs = ReedSolomon(k, n, field=a.field)
        self.rs.E, self.rs.G = e_mat, g
        gen = torch.Generator().manual_seed(rank + 1 if seed is None else seed)
        self.data = torch.randint(0, 256, (k, C), dtype=torch.uint8, generator=gen)
        self.parity = parity_bufs or [torch.zeros((self.p, C), dtype=torch.uint8) for _ in range(slots)]
        self.lanes = len(self.parity)
        self.outs = out_bufs or [torch.zeros((k, C), dtype=torch.uint8) for _ in range(self.lanes)]
        self.pool_dev = pool_dev
        self.bcast = False

    def flat_parity(self, slot: int) -> torch.Tensor:
        return self.parity[slot].reshape(-1)

    def piece_rows(self, slot: int) -> list[torch.Tensor]:
        return [self.parity[slot][i] for i in range(self.p)] + [self.outs[slot % self.lanes][i] for i in range(self.k)]

    def use_lane(self, slot: int) -> None:
        pass

    def step(self, i: int, slot: int) -> None:
        self.rs.encode(self.data, self.parity[slot])
        rows_t = self.pool_dev[i % self.pool_dev.shape[0]].clone()
        if self.bcast:  # the pattern comes from rank 0, as on the GPU path
            if self.rank != 0:
                rows_t.fill_(-1)
            dist.broadcast(rows_t, 0)
        rows = rows_t.tolist()
        stripe = [self.data[r] if r < self.k else self.parity[slot][r - self.k] for r in rows]
        self.rs.decode(stripe, rows, out=self.outs[slot % self.lanes])

    def sync(self) -> None:
        pass

    def reset(self) -> None:
        pass

    def verify(self) -> bool:
        want = _oracle_gemm(self.rs.E, self.data.numpy(), self.wide)
        return all(torch.equal(o, self.data) for o in self.outs) and all(
            np.array_equal(par.numpy(), want) for par in self.parity)


def make_work(a, k, n, C, e_mat, g, pool_dev, rank, dev, slots, **kw):
    if dev.type == "cuda":
        return GpuWorkload(a, k, n, C, e_mat, g, pool_dev, rank, dev, slots, **kw)
    return CpuWorkload(a, k, n, C, e_mat, g, pool_dev, rank, slots, **kw)


# ---- timing ----------------------------------------------------------------------------------
def _run_steps(work, xchg, steps: int) -> None:
    slots = len(work.parity)
    for i in range(steps):
        slot = i % slots
        work.use_lane(slot)
        xchg.wait(slot)  # the exchange that last read this slot's buffers is done
        work.step(i, slot)
        xchg.start(slot)
    xchg.drain()


def timed_loop(work, xchg, steps: int, world: int, dev, label: str) -> list[float]:
    """Seconds for `steps` steps, bracketed by barrier + synchronize on both sides, per rank (the
    headline takes the max over ranks)."""
    work.reset()
    with trace_range(f"bench/{label}"):
        if world > 1:
            dist.barrier()
        work.sync()
        t0 = time.perf_counter()
        _run_steps(work, xchg, steps)
        work.sync()
        if world > 1:
            dist.barrier()
        work.sync()
        elapsed = time.perf_counter() - t0
    return gather_over_ranks(elapsed, dev, world)


def gather_over_ranks(x: float, dev, world: int) -> list[float]:
    """x from every rank, in rank order (all_gather)."""
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    if world == 1:
        return [float(t.item())]
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [float(v.item()) for v in out]


def max_over_ranks(x: float, dev, world: int) -> float:
    return max(gather_over_ranks(x, dev, world))


def warm(work, xchg, steps: int, min_ms: float = 0.0) -> dict:
    """Untimed: first a pre-warm of local steps until `min_ms` has passed (no collectives: every
    rank draws its step's pattern from its own copy of the broadcast pool, so ranks need not agree on
    a count), then the `steps` warmup steps of the mode itself (with its traffic). The pre-warm is
    there because the GPU's clocks leave their idle state over the first ~100 ms of load: after 5
    warmup steps (~3 ms) the next 20 steps ran 4 % slower than after 300 (profiles/headline/r07_warm)."""
    info = {"steps": 0, "ms": 0.0}
    if min_ms > 0:
        bcast, work.bcast = work.bcast, False
        work.reset()
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < min_ms:
            _run_steps(work, _NoExchange(), 4)
            work.sync()
            info["steps"] += 4
        info["ms"] = round((time.perf_counter() - t0) * 1e3, 1)
        work.bcast = bcast
    work.reset()
    _run_steps(work, xchg, steps)
    work.sync()
    return info


class _NoExchange:
    def start(self, slot):
        pass

    def wait(self, slot):
        pass

    def drain(self):
        pass

    def verify(self, slot):
        return True


def e2e(a, k, n, C, rs: ReedSolomon, rows: list[int], work: GpuWorkload, dev, world: int) -> dict:
    """Reference-comparable timing on every rank at once: pinned host rows -> H2D -> GF-GEMM -> D2H
    (the native streaming pipeline, -s `a.streams`): encode, a decode that rebuilds the erased
    natives, and the reference's full decode (k x k inverse, all k natives into a [k, C] image)."""
    from gpu_rscode_amd._native import hip

    h = hip()
    p = n - k
    host = torch.empty((k, C), dtype=torch.uint8, pin_memory=True)
    host.copy_(work.data)
    par = torch.empty((p, C), dtype=torch.uint8, pin_memory=True)
    erased = [i for i in range(k) if i not in rows]
    rec = torch.empty((len(erased), C), dtype=torch.uint8, pin_memory=True)
    image = torch.empty((k, C), dtype=torch.uint8, pin_memory=True)  # the decoded file, contiguous
    dm_full = rs.decode_matrix(rows)
    enc_in = [host[j].data_ptr() for j in range(k)]
    enc_out = [par[i].data_ptr() for i in range(p)]
    dec_in = [host[r].data_ptr() if r < k else par[r - k].data_ptr() for r in rows]
    dec_out = [rec[i].data_ptr() for i in range(len(erased))]
    full_out = [image[i].data_ptr() for i in range(k)]
    emat = np.ascontiguousarray(rs.E).tobytes()
    dmat = np.ascontiguousarray(dm_full[erased]).tobytes()
    fmat = np.ascontiguousarray(dm_full).tobytes()
    h.prepare_pipeline([dev.index], k, max(p, k), C, a.streams, a.slice)

    def run(ins, outs, mat):
        return h.gemm_host([dev.index], ins, outs, mat, C, a.streams, a.slice, 0, False,
                           field_w=16 if work.wide else 8)["devices"][0]

    res = {}
    for name, ins, outs, mat in (("encode", enc_in, enc_out, emat), ("decode", dec_in, dec_out, dmat),
                                 ("decode_full", dec_in, full_out, fmat)):
        run(ins, outs, mat)  # warm (first DMA of fresh pinned pages)
        best = None
        for _ in range(3):
            if world > 1:
                dist.barrier()
            st = run(ins, outs, mat)
            t = max_over_ranks(st["ms_total"], dev, world)
            if best is None or t < best[0]:
                best = (t, st)
        res[name] = best
    ok = True
    for a0, b0 in _check_windows(C, even=work.wide):
        ok = ok and np.array_equal(par[:, a0:b0].numpy(), work.parity[0][:, a0:b0].cpu().numpy())
    ok = ok and torch.equal(rec, host[erased]) and torch.equal(image, host)
    stripe_bytes = k * C * world
    enc_ms, dec_ms, full_ms = res["encode"][0], res["decode"][0], res["decode_full"][0]
    both = 2 * stripe_bytes / ((enc_ms + dec_ms) / 1e3) / 1e9
    return {
        "encode_GBps": round(stripe_bytes / (enc_ms / 1e3) / 1e9, 3),
        "decode_GBps": round(stripe_bytes / (dec_ms / 1e3) / 1e9, 3),
        "decode_full_GBps": round(stripe_bytes / (full_ms / 1e3) / 1e9, 3),
        "encode_decode_GBps": round(both, 3),
        "vs_baseline_e2e": round(both / BASELINE_GBPS, 1),
        "encode_ms": round(enc_ms, 3), "decode_ms": round(dec_ms, 3), "decode_full_ms": round(full_ms, 3),
        "encode_ms_stream": round(res["encode"][1]["ms_stream"], 3),
        "decode_ms_stream": round(res["decode"][1]["ms_stream"], 3),
        "streams": a.streams, "slice_bytes": a.slice, "erased": len(erased), "verified": bool(ok),
        "what": "pinned host -> H2D -> GF-GEMM -> D2H per rank (own PCIe link), max over ranks; decode erases the "
                "first `erased` natives (src/unit-test.sh pattern) and reads the k survivors: decode writes the "
                "rebuilt natives (surviving natives stay in host memory), decode_full is the reference's shape "
                "(src/decode.cu:149-176: the whole k x k inverse, all k natives D2H into one contiguous image)",
    }


# ---- runs ------------------------------------------------------------------------------------
def weak_work(a, k, n, e_mat, g, pool_dev, rank, dev, has_pg):
    """The weak-scaling workload: every rank encodes and decodes its own a.bytes stripe."""
    C = (a.bytes + k - 1) // k
    if a.field == "gf65536":
        C += C % 2  # whole 16-bit symbols
    slots = 2 if has_pg else 1  # parity double-buffered while its exchange is in flight
    return make_work(a, k, n, C, e_mat, g, pool_dev, rank, dev, slots), C


def run_weak_mode(a, work, mode, world, dev, has_pg, steps, warmup, graph=False):
    """One barrier-bracketed timed loop of the weak workload with `mode`'s per-step traffic."""
    k, C = work.k, work.C
    slots = len(work.parity)
    xchg = ParityExchange([work.flat_parity(s) for s in range(slots)], mode if mode in ("owners", "root") else "none")
    work.bcast = has_pg and mode != "none"
    pre = warm(work, xchg, warmup, a.min_warmup_ms)
    if graph:
        work.graph_mode = True
        graphs = []
        for i in range(len(work.pool_dev)):
            gph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gph, stream=work.stream):
                work.step(i, 0)
            graphs.append(gph)
        torch.cuda.synchronize()
        step_fn = work.step
        work.step = lambda i, slot: graphs[i % len(graphs)].replay()  # noqa: E731
        per_rank = timed_loop(work, xchg, steps, world, dev, f"timed/weak/{mode}")
        work.step = step_fn
        work.graph_mode = False
        for j in range(steps):  # which pattern each decoder last solved (capture order differs)
            work._dec(j, 0).last_i = j
    else:
        per_rank = timed_loop(work, xchg, steps, world, dev, f"timed/weak/{mode}")
    ok = all(xchg.verify(s) for s in range(slots))
    return dict(elapsed=max(per_rank), per_rank=per_rank, steps=steps, ok=ok, sent=xchg.bytes_sent,
                recv=xchg.bytes_received, link=xchg.bytes_per_link, bytes=2 * k * C * world, prewarm=pre)


def run_strong(a, k, n, e_mat, g, pool_dev, rank, world, dev, has_pg, steps, warmup):
    """Strong scaling: ONE stripe of a.bytes column-sharded over the ranks (shard_range, the
    reference's split, src/encode.cu:368-381). Rank 0's shard computes in place inside its full
    rows, so the gather moves only the peers' pieces."""
    Ct = (a.bytes + k - 1) // k
    p = n - k
    lo, hi = shard_range(Ct, world, rank)
    widths = [b - a_ for a_, b in (shard_range(Ct, world, r) for r in range(world))]
    lanes = 1 if a.graph else max(1, a.lanes)
    slots = max(2 if (has_pg and a.gather == "step") else 1, lanes)
    fulls = None
    par_bufs = out_bufs = None
    if rank == 0 and a.gather != "none":
        mk = (lambda r: alloc_rows(r, Ct, dev)) if dev.type == "cuda" else (lambda r: torch.zeros((r, Ct), dtype=torch.uint8))
        full_par = [mk(p) for _ in range(slots)]
        full_out = [mk(k) for _ in range(lanes)]
        fulls = [[full_par[s][i] for i in range(p)] + [full_out[s % lanes][i] for i in range(k)] for s in range(slots)]
        par_bufs = [fp[:, :hi - lo] for fp in full_par]
        out_bufs = [fo[:, :hi - lo] for fo in full_out]
    work = make_work(a, k, n, hi - lo, e_mat, g, pool_dev, rank, dev, slots, parity_bufs=par_bufs,
                     out_bufs=out_bufs, seed=1000 + rank)
    slots = len(work.parity)
    gather = None
    if a.gather != "none":
        gather = StripeGather([work.piece_rows(s) for s in range(slots)], fulls, widths)
    xchg = gather if (gather is not None and a.gather == "step") else _NoExchange()
    work.bcast = has_pg
    pre = warm(work, xchg, warmup, a.min_warmup_ms)
    per_rank = timed_loop(work, xchg, steps, world, dev, f"timed/strong/{a.gather}")
    ok = all(xchg.verify(s) for s in range(slots))
    out = dict(elapsed=max(per_rank), per_rank=per_rank, steps=steps, ok=ok, bytes=2 * k * Ct, total_cols=Ct,
               prewarm=pre,
               widths=widths, gather=a.gather, link=gather.bytes_per_link if gather else 0,
               recv=gather.bytes_received if (gather and rank == 0) else 0)
    if a.gather == "end":
        if world > 1:
            dist.barrier()
        work.sync()
        t0 = time.perf_counter()
        gather.start(0)
        gather.drain()
        work.sync()
        gt = max(gather_over_ranks(time.perf_counter() - t0, dev, world))
        out.update(gather_ms=round(gt * 1e3, 3), gather_ok=gather.verify(0),
                   gather_GBps=round(gather.bytes_per_link * max(1, world - 1) / gt / 1e9, 3) if world > 1 else None)
        out["ok"] = out["ok"] and out["gather_ok"]
    return work, out


# ---- other BASELINE configs, each in a fresh child process (N = 1) ----------------------------
def _last_json(text: str) -> dict | None:
    for line in reversed(text.splitlines()):
        line = line.strip()
        if line.startswith("{"):
            try:
                return json.loads(line)
            except ValueError:
                return None
    return None


def run_config_child(a, preset: str, timeout_s: float) -> dict:
    """``bench.py --preset <preset>`` as a CHILD process (never an exec of this one) with its own
    timeout and process group; its one JSON line, condensed. A crash, a hang or a bad record gives
    ``{"error": ..., "rc": ...}`` — the caller's headline record is never touched."""
    device = PRESETS[preset].get("device", a.device)  # (a CPU preset runs on the CPU codec)
    cmd = [sys.executable, os.path.abspath(__file__), "--preset", preset, "--steps", str(a.config_steps),
           "--warmup", str(a.config_warmup), "--no-e2e", "--configs", "none", "--device", device,
           "--headline-budget", str(max(10.0, timeout_s - 5))]
    env = dict(os.environ, GFRS_CONFIG_CHILD=preset)
    t0 = time.perf_counter()
    try:
        proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env,
                                start_new_session=True)
    except OSError as ex:
        return {"error": f"could not start: {ex}", "rc": None}
    try:
        out, err = proc.communicate(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        try:
            os.killpg(proc.pid, 9)  # the child's own session: its group is exactly what we started
        except OSError:
            pass
        proc.communicate()
        return {"error": f"timed out after {timeout_s:.0f} s", "rc": None,
                "wall_s": round(time.perf_counter() - t0, 2)}
    wall = round(time.perf_counter() - t0, 2)
    rec = _last_json(out)
    if proc.returncode != 0 or rec is None or rec.get("value") is None:
        tail = (err or out or "").strip().splitlines()[-3:]
        return {"error": " | ".join(tail)[-400:] or "no record", "rc": proc.returncode, "wall_s": wall,
                **({"verified": rec.get("verified")} if rec else {})}
    cfg = rec.get("config", {})
    return {"metric": rec.get("metric"), "value": rec.get("value"), "unit": rec.get("unit"),
            "ms_per_step": rec.get("ms_per_step"), "verified": rec.get("verified"), "steps": rec.get("steps"),
            "warmup": rec.get("warmup"), "dtype": rec.get("dtype"), "model": cfg.get("model"),
            "global_batch": cfg.get("global_batch"), "engine": cfg.get("engine"), "rc": proc.returncode,
            "wall_s": wall}


def run_configs(a, rec: dict) -> None:
    """Time each of ``a.configs`` in its own child process (after the headline is verified and held
    in ``rec``) and embed the condensed records under ``rec["configs"]``."""
    if not a.configs:
        return
    deadline = time.perf_counter() + a.configs_budget
    rec["configs"] = {}
    for preset in a.configs:
        left = deadline - time.perf_counter()
        if left < 10:
            rec["configs"][preset] = {"skipped": f"--configs-budget ({a.configs_budget:g} s) spent"}
            continue
        rec["configs"][preset] = run_config_child(a, preset, min(75.0, left))
    rec["configs_what"] = ("other BASELINE configs, each timed by bench.py --preset P in a fresh child process "
                           "after the headline (steps / warmup as listed; verified like the headline)")


def _maybe_child_fault(preset: str) -> None:
    """Test hook: GFRS_CONFIG_FAULT=<preset>:crash|hang makes that --configs child fail."""
    spec = os.environ.get("GFRS_CONFIG_FAULT", "")
    if os.environ.get("GFRS_CONFIG_CHILD") != preset or ":" not in spec:
        return
    which, kind = spec.split(":", 1)
    if which != preset:
        return
    if kind == "hang":
        time.sleep(3600)
    os._exit(7)


# ---- failure isolation (N > 1) ---------------------------------------------------------------
class Emitter:
    """Prints the ONE JSON record exactly once (rank 0), from the main thread or from a watchdog."""

    def __init__(self, rank: int):
        self.rank = rank
        self.lock = threading.Lock()
        self.done = False

    def emit(self, rec: dict) -> bool:
        with self.lock:
            if self.done:
                return False
            self.done = True
            if self.rank == 0:
                sys.stdout.write(json.dumps(rec) + "\n")
            sys.stdout.flush()
            sys.stderr.flush()
            return True


class Watchdog:
    """Deadline for a stretch of collectives that may hang (an RCCL kernel whose peer never joins
    does not raise). When it expires, `on_expire()` runs on the watchdog thread (rank 0 prints the
    record it holds, with the stretch marked as timed out) and the process ends with `code` — no
    re-exec, no further collectives. Every rank runs one with the same budget, so all ranks leave."""

    def __init__(self, budget_s: float, on_expire, code: int = 0):
        self.budget_s, self.on_expire, self.code = budget_s, on_expire, code
        self.timer = threading.Timer(budget_s, self._fire)
        self.timer.daemon = True

    def _fire(self) -> None:
        try:
            self.on_expire()
        finally:
            os._exit(self.code)

    def __enter__(self):
        self.timer.start()
        return self

    def __exit__(self, *exc):
        self.timer.cancel()
        return False


def _err(e: BaseException) -> str:
    return f"{type(e).__name__}: {e}"[:500]


def agree(ok: bool, dev, world: int) -> list[int]:
    """Every rank's status after a comparison mode (1 ok, 0 failed verification), in rank order."""
    if world == 1:
        return [1 if ok else 0]
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [int(x.item()) for x in out]


# ---- main ------------------------------------------------------------------------------------
def gbps_of(r) -> float:
    return r["bytes"] / (r["elapsed"] / r["steps"]) / 1e9


def mode_entry(r, rank) -> dict:
    """value_by_comm entry of a timed weak mode: rate, the busiest xGMI link's bytes per step and
    the rate the measured step implies for it (a lower bound on what the link sustained; when the
    step is link-bound, its rate)."""
    return {"GBps": round(gbps_of(r), 3), "ms_per_step": round(r["elapsed"] / r["steps"] * 1e3, 4),
            "steps": r["steps"], "bytes_sent_per_rank_step": r["sent"],
            "bytes_recv_rank0_step": r["recv"] if rank == 0 else None,
            "busiest_link_bytes_per_step": r["link"],
            "busiest_link_GBps_implied": round(r["link"] / (r["elapsed"] / r["steps"]) / 1e9, 4),
            "step_ms_by_rank": [round(x / r["steps"] * 1e3, 4) for x in r["per_rank"]],
            "verified": r["ok"]}


def strong_entry(a, strong, rank) -> dict:
    return {"GBps": round(gbps_of(strong), 3), "ms_per_step": round(strong["elapsed"] / strong["steps"] * 1e3, 4),
            "steps": strong["steps"], "stripe_bytes": a.bytes, "shard_cols": strong["widths"],
            "gather": strong["gather"], "busiest_link_bytes_per_step": strong["link"],
            "bytes_recv_rank0": strong["recv"] if rank == 0 else None, "verified": strong["ok"],
            "step_ms_by_rank": [round(x / strong["steps"] * 1e3, 4) for x in strong["per_rank"]],
            **{kk: strong[kk] for kk in ("gather_ms", "gather_GBps") if kk in strong}}


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    a = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (a.gpus or 1) > 1:
        return launch(a.gpus, argv)  # parent: no GPU call before (or after) this
    world = int(env_world or "1")
    _maybe_child_fault(a.preset)
    if a.gpus is not None and a.gpus != world:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.device == "cuda":
        if a.rehearsal:  # (device_count does not initialise the GPU)
            local %= max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    has_pg = world > 1 or a.force_pg
    emitter = Emitter(rank)
    k, n = a.k, a.n
    # The headline's own deadline: setup + warmup + the timed loop + its verification. A hang here
    # leaves no number to save; the record says where it stopped instead of the driver's timeout.
    stage = {"at": "setup"}

    def headline_expired():
        emitter.emit({"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": world, "steps": a.steps,
                      "warmup": a.warmup, "higher_is_better": True, "verified": False,
                      "error": f"headline timed out after {a.headline_budget:g} s during {stage['at']}"})

    with Watchdog(a.headline_budget, headline_expired, code=3):
        if has_pg:
            kw = {"device_id": dev} if a.pg_backend == "nccl" else {}
            if world == 1 and "MASTER_PORT" not in os.environ:
                kw.update(init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
            # bounded: a lost peer raises (gloo) or is aborted by the RCCL watchdog after this long;
            # the bench's own watchdogs (shorter) print the record first
            dist.init_process_group(a.pg_backend, timeout=datetime.timedelta(seconds=a.pg_timeout), **kw)
            if dist.get_world_size() != world:
                raise SystemExit("process group size does not match WORLD_SIZE")
        if a.graph and has_pg:
            raise SystemExit("--graph is single-GPU only, without a process group (per-step RCCL traffic)")

        # ---- setup: E and the erasure-pattern pool come from rank 0 (RCCL broadcast) ---------
        rs = ReedSolomon(k, n, field=a.field)
        wide = rs.wide
        pool = erasure_pool(k, n, a.erasures, rs)
        # (GF(2^16): E travels as int16 words — the collectives have no uint16)
        e_t = torch.from_numpy(rs.E.astype("<u2").view(np.int16) if wide else rs.E.copy()).to(dev)
        pool_t = torch.tensor(pool, dtype=torch.int32, device=dev)
        if has_pg:
            dist.broadcast(e_t, 0)
            dist.broadcast(pool_t, 0)
        e_mat = e_t.cpu().numpy()
        if wide:
            e_mat = e_mat.view("<u2").astype(np.uint16)
            rs.E, rs.G = e_mat, np.vstack([np.eye(k, dtype=np.uint16), e_mat])
        else:
            rs.E, rs.G = e_mat, gf.GF256.generator(e_mat)

        # ---- the headline: timed, verified and reduced before anything else runs --------------
        head_strong = a.scaling == "strong"
        head_mode = a.comm if has_pg else "none"
        if head_strong:
            stage["at"] = "strong headline"
            work, head = run_strong(a, k, n, e_mat, rs.G, pool_t, rank, world, dev, has_pg, a.steps, a.warmup)
            C = work.C
        else:
            stage["at"] = f"weak/{head_mode} headline"
            work, C = weak_work(a, k, n, e_mat, rs.G, pool_t, rank, dev, has_pg)
            head = run_weak_mode(a, work, head_mode, world, dev, has_pg, a.steps, a.warmup, graph=a.graph)
        stage["at"] = "headline verification"
        ok = work.verify() and head["ok"]
        okt = torch.tensor([1 if ok else 0], device=dev)
        if world > 1:
            dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = bool(okt.item())
        rec = headline_record(a, k, n, C, world, rank, dev, has_pg, work, head, head_strong, head_mode, ok)

    # ---- comparison modes: each on its own, after the headline is safe ----------------------
    # A mode that raises is recorded as {"error": ...}; a mode that hangs is cut off by the
    # watchdog, which prints the record held so far. After any failure no further collective is
    # issued (the group may be out of step): rank 0 prints and every rank leaves.
    # Order: least collective risk first (e2e: own PCIe link + barriers; none: no traffic; owners:
    # one all_to_all), the point-to-point gathers (strong, root) last.
    compare = has_pg and not a.no_compare
    todo = []
    if dev.type == "cuda" and not a.no_e2e and not head_strong:
        todo.append(("e2e", None))
    if compare and not head_strong:
        todo += [("weak", m) for m in ("none", "owners", "bcast") if m != head_mode]
        todo.append(("strong", a.gather))
        if head_mode != "root":
            todo.append(("weak", "root"))
    done = {"n": 0}

    def mark_rest(reason: str, start: int, failed: int | None = None):
        for j in range(start, len(todo)):
            kind, m = todo[j]
            _store(rec, kind, m, {"error": reason} if j == failed else {"skipped": reason})

    def compare_expired():
        cur = todo[done["n"]] if done["n"] < len(todo) else None
        mark_rest(f"timed out ({a.compare_budget:g} s budget for the comparison modes)", done["n"], done["n"])
        if cur is not None:
            mark_rest(f"after {cur[0]}/{cur[1]} timed out", done["n"] + 1)
        rec["comparisons_complete"] = False
        emitter.emit(rec)

    clean = True
    with Watchdog(a.compare_budget, compare_expired, code=0 if ok else 1):
        for i, (kind, m) in enumerate(todo):
            done["n"] = i
            try:
                if kind == "weak":
                    r = run_weak_mode(a, work, m, world, dev, has_pg, min(a.steps, 20), 2)
                    r["ok"] = r["ok"] and work.verify()
                    entry = mode_entry(r, rank)
                elif kind == "strong":
                    swork, r = run_strong(a, k, n, e_mat, rs.G, pool_t, rank, world, dev, has_pg, min(a.steps, 20), 2)
                    r["ok"] = r["ok"] and swork.verify()
                    del swork
                    entry = strong_entry(a, r, rank)
                else:
                    # the reference's worst case (src/unit-test.sh: keep the last k chunks): the first
                    # `erasures` natives are lost, so every one of them is rebuilt and copied back
                    e = min(a.erasures, k, n - k)
                    entry = e2e(a, k, n, C, rs, list(range(e, k)) + list(range(k, k + e)), work, dev, world)
                    r = {"ok": entry["verified"]}
                status = agree(r["ok"], dev, world)
            except Exception as ex:  # noqa: BLE001 — recorded, then this rank stops issuing collectives
                _store(rec, kind, m, {"error": f"rank {rank}: {_err(ex)}"})
                print(f"bench.py rank {rank}: {kind}/{m} failed: {_err(ex)}", file=sys.stderr, flush=True)
                mark_rest(f"after {kind}/{m} failed", i + 1)
                clean = False
                break
            if kind == "weak" or kind == "strong":
                entry["verified"] = entry["verified"] and min(status) == 1
                if min(status) == 0:
                    entry["failed_ranks"] = [r_ for r_, s_ in enumerate(status) if s_ == 0]
            _store(rec, kind, m, entry)
        else:
            done["n"] = len(todo)
    if compare:
        rec["comparisons_complete"] = clean
    if world == 1 and clean:
        run_configs(a, rec)
    emitter.emit(rec)
    if has_pg and clean:
        # (the record is out; a teardown that hangs must not hold the job: leave after 60 s)
        with Watchdog(60.0, lambda: None, code=0 if ok else 1):
            dist.destroy_process_group()
    if not clean:  # the group may be out of step: leave without another collective
        os._exit(0 if ok else 1)
    return 0 if ok else 1


def _store(rec: dict, kind: str, m, entry: dict) -> None:
    if kind == "weak":
        rec.setdefault("value_by_comm", {})[m] = entry
        if m == "none" and "GBps" in entry:
            rec["value_no_comm"] = entry["GBps"]
    elif kind == "strong":
        rec["strong"] = entry
        if "GBps" in entry:
            rec["value_strong"] = entry["GBps"]
    else:
        rec["e2e"] = entry
        rec["vs_baseline"] = entry.get("vs_baseline_e2e") if entry.get("verified") else None


def headline_record(a, k, n, C, world, rank, dev, has_pg, work, head, head_strong, head_mode, ok) -> dict:
    ms = head["elapsed"] / head["steps"] * 1e3
    value = gbps_of(head)
    metric = METRIC
    if a.preset != "k10n14" or a.bytes != PRESETS["k10n14"]["bytes"] or head_strong or a.field != "gf256":
        per = "in total, one stripe sharded over the GPUs" if head_strong else "per GPU"
        fld = ", GF(2^16)" if a.field == "gf65536" else ""
        metric = f"encode+decode throughput (GB/s) at k={k},n={n}{fld} on {a.bytes / 2**30:.3g} GiB {per}"
    comm_desc = {"bcast": "rank 0 RCCL-broadcasts the step's erasure pattern; parity and decoded rows stay in "
                          "each GPU's HBM (as at N = 1)",
                 "owners": "pattern broadcast + parity all_to_all to chunk owners over RCCL/xGMI",
                 "root": "pattern broadcast + parity gather to rank 0 over RCCL/xGMI (grouped send/recv)",
                 "none": "no per-step traffic (each rank draws the pattern itself)"}
    if head_strong:
        parallelism = f"dp{world} strong (one {k}-row stripe column-sharded, gather {a.gather})"
        comm_what = {"step": "pattern broadcast + parity and decoded natives gathered into rank 0 every step",
                     "end": "pattern broadcast; parity and decoded natives gathered into rank 0 once, after the "
                            "timed loop (timed on its own: strong.gather_ms)",
                     "none": "pattern broadcast only"}[a.gather] if has_pg else "none (one GPU)"
    else:
        parallelism = f"dp{world} weak (stripe per rank, E + pattern pool RCCL-broadcast)"
        comm_what = comm_desc[head_mode]
    step_ms = [x / head["steps"] * 1e3 for x in head["per_rank"]]
    rec = {
        "metric": metric,
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "prewarm": {**head.get("prewarm", {}), "min_ms": a.min_warmup_ms,
                    "what": "untimed local steps (no collectives) run before the warmup steps until min_ms "
                            "passed: clocks leave idle over the first ~100 ms of load"},
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "strong" if head_strong else "weak",
        # like for like with the reference's PCIe-inclusive MB/s (doc/design.tex:482-500): filled from the
        # e2e timing below (_store); the device-resident ratio is vs_baseline_device
        "vs_baseline": None,
        "vs_baseline_device": round(value / BASELINE_GBPS, 1),
        "dtype": "uint16 (GF(2^16) symbols)" if a.field == "gf65536" else "uint8 (GF(2^8) symbols)",
        "data": "synthetic (device-generated random bytes)" if dev.type == "cuda" else "synthetic (host random bytes)",
        "config": {"model": (f"RS(k={k},n={n}) reference Vandermonde, GF(2^16) poly 0x1100B" if a.field == "gf65536"
                             else f"RS(k={k},n={n}) reference Vandermonde, GF(2^8) poly 0x11D"),
                   "global_batch": (f"{a.bytes} B in total ({k} x {C} B columns per rank shard)" if head_strong
                                    else f"{a.bytes} B per GPU ({k} x {C} B chunks)"),
                   "seq_len": C, "parallelism": parallelism,
                   "comm": ("strong/" + a.gather) if head_strong else head_mode, "comm_what": comm_what,
                   "erasures": a.erasures,
                   "decode_invert": ("device-built plan per step: pattern check + systematic e x (e+k) Gauss-Jordan "
                                     "+ descriptor rows/tables" if dev.type == "cuda"
                                     else "host row-pivoted Gauss-Jordan (cached per pattern)"),
                   "engine": getattr(getattr(work, "enc", [None])[0], "engine", "cpu"), "graph": bool(a.graph),
                   "preset": a.preset, "device": dev.type, "process_group": bool(has_pg),
                   "pg_backend": a.pg_backend if has_pg else None,
                   "rehearsal": (f"{world} ranks sharing {torch.cuda.device_count()} GPU(s) over gloo: a code-path "
                                 "check, not a scaling number") if (a.rehearsal and has_pg) else None,
                   "bcast_ahead": a.bcast_ahead if (has_pg and dev.type == "cuda") else None},
        "verified": ok,
        # per-rank step time of the headline loop (each rank's own clock between the barriers): a
        # straggler shows as the max; the headline uses the max
        "step_ms_by_rank": {"min": round(min(step_ms), 4), "max": round(max(step_ms), 4),
                            "per_rank": [round(x, 4) for x in step_ms]},
        "vs_baseline_what": "vs_baseline = e2e.vs_baseline_e2e: pinned host -> GPU -> host encode + decode "
                            "throughput / the reference's nearest published point, which is PCIe-inclusive "
                            "(null if the e2e timing did not run); vs_baseline_device = device-resident value / "
                            "that same point (not like for like)",
        "baseline": {"gbps": round(BASELINE_GBPS, 4), "source": "k=8,n=11 1.1 GB Tesla C2050 (nearest published)"},
    }
    if has_pg and not head_strong:
        rec["headline_why"] = ("weak scaling with the parity left in each GPU's HBM, as the N = 1 number does; the "
                               "per-step parity movement over xGMI (value_by_comm.owners / .root) and the "
                               "reference's one-stripe strong scaling (value_strong) are timed after it, each "
                               "on its own (a failing comparison mode is recorded, never the headline lost)")
        rec["value_by_comm"] = {head_mode: mode_entry(head, rank)}
    if head_strong:
        rec["value_strong"] = round(value, 3)
        rec["strong"] = strong_entry(a, head, rank)
    return rec


if __name__ == "__main__":
    sys.exit(main())
