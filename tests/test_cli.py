"""Python CLI: single-process (CPU backend) and torchrun --dist mode over gloo (world size 2)."""
import os
import socket
import subprocess
import sys

import pytest

from gpu_rscode_amd.utils import fileformat as ff

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _py(args, cwd, env=None):
    e = dict(os.environ, PYTHONPATH=ROOT, **(env or {}))
    return subprocess.run([sys.executable, "-m", "gpu_rscode_amd", *args], cwd=cwd, capture_output=True, text=True,
                          timeout=300, env=e)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_python_cli_cpu_roundtrip(tmp_path):
    payload = os.urandom(123_457)
    (tmp_path / "f.bin").write_bytes(payload)
    r = _py(["-k", "4", "-n", "6", "-e", "f.bin", "--backend", "cpu", "--matrix", "cauchy"], tmp_path)
    assert r.returncode == 0, r.stderr
    ff.write_conf(str(tmp_path / "conf"), ["_0_f.bin", "_3_f.bin", "_4_f.bin", "_5_f.bin"])
    r = _py(["-d", "-i", "f.bin", "-c", "conf", "-o", "o.bin", "--backend", "cpu"], tmp_path)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "o.bin").read_bytes() == payload


@pytest.mark.parametrize("w", [8, 16])
def test_torchrun_dist_cli_matches_single_process(tmp_path, w):
    payload = os.urandom(3 * 4096 * 10 + 999)
    d1, d2 = tmp_path / "dist", tmp_path / "single"
    d1.mkdir()
    d2.mkdir()
    (d1 / "f.bin").write_bytes(payload)
    (d2 / "f.bin").write_bytes(payload)
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    base = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
            "--master-addr=127.0.0.1", f"--master-port={_port()}", "-m", "gpu_rscode_amd", "--dist"]
    r = subprocess.run(base + ["-k", "10", "-n", "14", "-w", str(w), "-e", "f.bin"], cwd=d1, capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    r = _py(["-k", "10", "-n", "14", "-w", str(w), "-e", "f.bin", "--backend", "cpu"], d2)
    assert r.returncode == 0, r.stderr
    for i in range(14):
        assert (d1 / f"_{i}_f.bin").read_bytes() == (d2 / f"_{i}_f.bin").read_bytes(), i
    # the METADATA (matrix and the CRCs combined from both ranks' shards) is the single process's
    assert (d1 / "f.bin.METADATA").read_bytes() == (d2 / "f.bin.METADATA").read_bytes()
    ff.write_conf(str(d1 / "conf"), [f"_{i}_f.bin" for i in (1, 2, 3, 5, 6, 8, 10, 11, 12, 13)])
    base[6] = f"--master-port={_port()}"
    r = subprocess.run(base + ["-d", "-i", "f.bin", "-c", "conf", "-o", "o.bin"], cwd=d1, capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert (d1 / "o.bin").read_bytes() == payload


def test_torchrun_dist_cli_split_survivor_check(tmp_path):
    """The multi-GPU decode checks its survivors split over the ranks: each rank CRCs only its
    column shard of every listed chunk, and rank 0 combines the CRCs and picks. A chunk corrupted
    only inside the last rank's shard, and a chunk that is missing, are both skipped (3 ranks,
    gloo), and the file comes back byte-exact."""
    payload = os.urandom(5 * 4096 * 10 + 777)
    (tmp_path / "f.bin").write_bytes(payload)
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = _py(["-k", "10", "-n", "14", "-e", "f.bin", "--backend", "cpu"], tmp_path)
    assert r.returncode == 0, r.stderr
    chunk = (tmp_path / "_1_f.bin").read_bytes()
    bad = bytearray(chunk)
    bad[len(bad) - 3] ^= 0x21  # last columns: the last rank's shard only
    (tmp_path / "_1_f.bin").write_bytes(bytes(bad))
    os.remove(tmp_path / "_4_f.bin")
    ff.write_conf(str(tmp_path / "conf"), [f"_{i}_f.bin" for i in range(14)])
    base = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
            "--master-addr=127.0.0.1", f"--master-port={_port()}", "-m", "gpu_rscode_amd", "--dist"]
    r = subprocess.run(base + ["-d", "-i", "f.bin", "-c", "conf", "-o", "o.bin"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert (tmp_path / "o.bin").read_bytes() == payload


def test_torchrun_dist_cli_windows_world3_and_stale_outputs(tmp_path):
    """3 ranks walking their shards in 4 KiB windows (uneven shard sizes, so some ranks run out of
    columns while the window collective continues), over stale, longer chunk / output files."""
    payload = os.urandom(7 * 4096 * 12 + 4321)
    d1, d2 = tmp_path / "dist", tmp_path / "single"
    d1.mkdir()
    d2.mkdir()
    (d1 / "f.bin").write_bytes(payload)
    (d2 / "f.bin").write_bytes(payload)
    for i in range(16):  # stale chunk files from an older, longer encode
        (d1 / f"_{i}_f.bin").write_bytes(b"\xee" * (len(payload) // 4))
    (d1 / "o.bin").write_bytes(b"\xee" * (2 * len(payload)))
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    base = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
            "--master-addr=127.0.0.1", f"--master-port={_port()}", "-m", "gpu_rscode_amd", "--dist",
            "--window", "4096", "--no-sync"]
    r = subprocess.run(base + ["-k", "12", "-n", "16", "-e", "f.bin"], cwd=d1, capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    r = _py(["-k", "12", "-n", "16", "-e", "f.bin", "--backend", "cpu"], d2)
    assert r.returncode == 0, r.stderr
    for i in range(16):
        assert (d1 / f"_{i}_f.bin").read_bytes() == (d2 / f"_{i}_f.bin").read_bytes(), i
    ff.write_conf(str(d1 / "conf"), [f"_{i}_f.bin" for i in (0, 2, 3, 4, 6, 7, 8, 10, 12, 13, 14, 15)])
    base[6] = f"--master-port={_port()}"
    r = subprocess.run(base + ["-d", "-i", "f.bin", "-c", "conf", "-o", "o.bin"], cwd=d1, capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert (d1 / "o.bin").read_bytes() == payload


def test_torchrun_dist_cli_bounded_host_memory(tmp_path):
    """The distributed CLI streams a file much larger than its window without holding it: the peak
    RSS of any rank stays within a fixed margin of a bare `import torch, gpu_rscode_amd` process
    (a whole-file read on rank 0 would add the file size, 256 MiB, to it)."""
    import resource

    size = 256 << 20
    with open(tmp_path / "f.bin", "wb") as f:
        block = os.urandom(1 << 20)
        for i in range(size >> 20):
            f.write(block[i:] + block[:i])
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-c", "import torch, gpu_rscode_amd, gpu_rscode_amd._native as n; n.cpu()"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    base_kib = resource.getrusage(resource.RUSAGE_CHILDREN).ru_maxrss
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", "-m", "gpu_rscode_amd", "--dist",
           "--window", str(4 << 20), "--no-sync"]
    r = subprocess.run(cmd + ["-k", "4", "-n", "6", "-e", "f.bin"], cwd=tmp_path, capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    ff.write_conf(str(tmp_path / "conf"), ["_0_f.bin", "_2_f.bin", "_4_f.bin", "_5_f.bin"])
    cmd[6] = f"--master-port={_port()}"
    r = subprocess.run(cmd + ["-d", "-i", "f.bin", "-c", "conf", "-o", "o.bin"], cwd=tmp_path, capture_output=True,
                       text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    peak_kib = resource.getrusage(resource.RUSAGE_CHILDREN).ru_maxrss
    with open(tmp_path / "f.bin", "rb") as a, open(tmp_path / "o.bin", "rb") as b:
        while True:
            x, y = a.read(1 << 24), b.read(1 << 24)
            assert x == y
            if not x:
                break
    assert peak_kib - base_kib < 160 * 1024, (base_kib, peak_kib)


def test_torchrun_dist_cli_rank_failure_exits_in_bounded_time(tmp_path):
    """World 3, rank 1 fails inside its shard (GFRS_DIST_FAULT_RANK): it exits non-zero without
    another collective, the job ends non-zero well inside the process-group timeout, and rank 0's
    METADATA is never written (no half-encoded stripe looks complete)."""
    import time

    payload = os.urandom(5 * 4096 * 9 + 77)
    (tmp_path / "f.bin").write_bytes(payload)
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               GFRS_DIST_FAULT_RANK="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", "-m", "gpu_rscode_amd", "--dist",
           "--pg-timeout", "60", "-k", "8", "-n", "11", "-e", "f.bin"]
    t0 = time.monotonic()
    r = subprocess.run(cmd, cwd=tmp_path, capture_output=True, text=True, timeout=240, env=env)
    took = time.monotonic() - t0
    assert r.returncode != 0 and "injected fault" in r.stderr, r.stderr[-3000:]
    assert took < 120, took
    assert not (tmp_path / "f.bin.METADATA").exists()
    # and a decode whose rank fails after the survivor broadcast
    env.pop("GFRS_DIST_FAULT_RANK")
    cmd[6] = f"--master-port={_port()}"
    r = subprocess.run(cmd, cwd=tmp_path, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    ff.write_conf(str(tmp_path / "conf"), [f"_{i}_f.bin" for i in range(3, 11)])
    env["GFRS_DIST_FAULT_RANK"] = "2"
    dcmd = cmd[:10] + ["--pg-timeout", "60", "-d", "-i", "f.bin", "-c", "conf", "-o", "o.bin"]
    dcmd[6] = f"--master-port={_port()}"
    t0 = time.monotonic()
    r = subprocess.run(dcmd, cwd=tmp_path, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode != 0 and "injected fault" in r.stderr and time.monotonic() - t0 < 120, r.stderr[-3000:]


@pytest.mark.parametrize("stop_rank", [0, 1])
def test_torchrun_dist_cli_resumes_after_a_shard_crash(tmp_path, stop_rank):
    """A --dist job whose rank `stop_rank` stops after one window (--stop-after: a simulated crash)
    fails without a METADATA; the re-run keeps the chunk files (no truncation), resumes the stopped
    shard from its checkpoint and every finished shard at its end, and the stripe comes out
    byte-exact, with every checkpoint gone. The same for a decode into an output file. (Round 5's
    rank 0 re-created the outputs zero-filled, so the columns a shard had checkpointed became zeros.)"""
    payload = os.urandom(4 * 4096 * 10 + 999)
    d1, d2 = tmp_path / "dist", tmp_path / "single"
    d1.mkdir()
    d2.mkdir()
    (d1 / "f.bin").write_bytes(payload)
    (d2 / "f.bin").write_bytes(payload)
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")

    def job(args):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
               "--master-addr=127.0.0.1", f"--master-port={_port()}", "-m", "gpu_rscode_amd", "--dist",
               "--window", "4096", "--pg-timeout", "60", *args]
        return subprocess.run(cmd, cwd=d1, capture_output=True, text=True, timeout=300, env=env)

    enc = ["-k", "10", "-n", "14", "-e", "f.bin"]
    r = job(enc + ["--stop-after", "1", "--stop-rank", str(stop_rank)])
    assert r.returncode != 0 and "--stop-after" in r.stderr, r.stderr[-3000:]
    assert not (d1 / "f.bin.METADATA").exists()
    assert any(x.startswith("f.bin.PROGRESS.") for x in os.listdir(d1))
    r = job(enc)
    assert r.returncode == 0, r.stderr[-3000:]
    assert _py(enc + ["--backend", "cpu"], d2).returncode == 0
    for name in [f"_{i}_f.bin" for i in range(14)] + ["f.bin.METADATA"]:
        assert (d1 / name).read_bytes() == (d2 / name).read_bytes(), name
    assert not [x for x in os.listdir(d1) if ".PROGRESS" in x]

    # a chunk lost between the crash and the re-run: it is re-created, so no checkpoint is trusted
    r = job(enc + ["--stop-after", "1", "--stop-rank", str(stop_rank)])
    assert r.returncode != 0
    os.remove(d1 / "_12_f.bin")
    r = job(enc)
    assert r.returncode == 0, r.stderr[-3000:]
    for name in [f"_{i}_f.bin" for i in range(14)] + ["f.bin.METADATA"]:
        assert (d1 / name).read_bytes() == (d2 / name).read_bytes(), name

    ff.write_conf(str(d1 / "conf"), [f"_{i}_f.bin" for i in (0, 2, 3, 4, 6, 7, 10, 11, 12, 13)])
    dec = ["-d", "-i", "f.bin", "-c", "conf", "-o", "o.bin"]
    r = job(dec + ["--stop-after", "1", "--stop-rank", str(stop_rank)])
    assert r.returncode != 0, r.stderr[-3000:]
    r = job(dec)
    assert r.returncode == 0, r.stderr[-3000:]
    assert (d1 / "o.bin").read_bytes() == payload
    assert not [x for x in os.listdir(d1) if ".PROGRESS" in x]


def test_dist_ipc_env_is_set_before_torch_distributed(tmp_path):
    """`python -m gpu_rscode_amd --dist` reaches torch.distributed with HSA_ENABLE_IPC_MODE_LEGACY=0
    already in the environment (the HIP runtime reads it once, at initialisation), even when the
    caller's environment lacks it: the package sets it before its own `import torch`."""
    probe = ("import os, sys\n"
             "import torch.distributed as d\n"
             "seen = []\n"
             "orig = d.init_process_group\n"
             "def spy(*a, **k):\n"
             "    seen.append(os.environ.get('HSA_ENABLE_IPC_MODE_LEGACY'))\n"
             "    raise SystemExit(7 if seen[0] == '0' else 8)\n"
             "d.init_process_group = spy\n"
             "from gpu_rscode_amd.utils.cli import main\n"
             "main(['--dist', '-k', '2', '-n', '3', '-e', 'f.bin'])\n")
    env = {k: v for k, v in os.environ.items() if k != "HSA_ENABLE_IPC_MODE_LEGACY"}
    env.update(PYTHONPATH=ROOT, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_port()), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    (tmp_path / "f.bin").write_bytes(b"x" * 100)
    r = subprocess.run([sys.executable, "-c", probe], cwd=tmp_path, capture_output=True, text=True, timeout=120,
                       env=env)
    assert r.returncode == 7, (r.returncode, r.stderr[-2000:])
    # the package sets it before ITS first `import torch` (torch's HIP runtime may initialise from then on)
    order = ("import builtins, os, sys\n"
             "real = builtins.__import__\n"
             "seen = []\n"
             "def imp(name, *a, **k):\n"
             "    if name == 'torch' and not seen:\n"
             "        seen.append(os.environ.get('HSA_ENABLE_IPC_MODE_LEGACY'))\n"
             "    return real(name, *a, **k)\n"
             "builtins.__import__ = imp\n"
             "import gpu_rscode_amd\n"
             "sys.exit(0 if seen == ['0'] else 9)\n")
    r = subprocess.run([sys.executable, "-c", order], cwd=tmp_path, capture_output=True, text=True, timeout=120,
                       env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    # and a process whose HIP is already up without it is refused an RCCL group (not a late failure)
    from gpu_rscode_amd.parallel import dist as pdist

    saved = os.environ.pop("HSA_ENABLE_IPC_MODE_LEGACY", None)
    try:
        import torch

        orig = torch.cuda.is_initialized
        torch.cuda.is_initialized = lambda: True
        try:
            with pytest.raises(RuntimeError, match="HSA_ENABLE_IPC_MODE_LEGACY"):
                pdist.ensure_ipc_env("nccl")
        finally:
            torch.cuda.is_initialized = orig
        pdist.ensure_ipc_env("gloo")  # (gloo needs no IPC)
        pdist.ensure_ipc_env("nccl")  # HIP not up: set in time
        assert os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    finally:
        if saved is not None:
            os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = saved
