"""Host sanitizer run: the CPU codec, METADATA/conf parsing and the file codec under
ASan + UBSan (bin/CPU-RS-asan, built by `make -C csrc sanitize`). Exercises odd sizes, every
erasure subset at (4,6), wide stripes, CRC rejection and malformed inputs."""
import fcntl
import itertools
import os
import subprocess

import pytest

from gpu_rscode_amd._build import CSRC, binary
from gpu_rscode_amd.utils import fileformat as ff


@pytest.fixture(scope="module")
def exe():
    # one build at a time: parallel test workers (pytest -n) would otherwise relink the binary
    # while another worker runs it
    with open(os.path.join(str(CSRC), ".sanitize.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        r = subprocess.run(["make", "-C", str(CSRC), "-j8", "sanitize"], capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        pytest.skip(f"sanitizer build unavailable: {r.stderr[-500:]}")
    return str(binary("CPU-RS-asan"))


def _run(exe, args, cwd):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe, *args], cwd=cwd, capture_output=True, text=True, timeout=300, env=env)
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
    return r


def test_asan_roundtrips(exe, tmp_path):
    payload = os.urandom(100_003)
    (tmp_path / "f.bin").write_bytes(payload)
    assert _run(exe, ["-k", "4", "-n", "6", "-e", "f.bin", "--mul", "logexp3"], tmp_path).returncode == 0
    for rows in itertools.combinations(range(6), 4):
        ff.write_conf(str(tmp_path / "c"), [f"_{r}_f.bin" for r in rows])
        assert _run(exe, ["-d", "-i", "f.bin", "-c", "c", "-o", "o"], tmp_path).returncode == 0
        assert (tmp_path / "o").read_bytes() == payload


def test_asan_wide_and_malformed(exe, tmp_path):
    payload = os.urandom(12_345)
    (tmp_path / "w.bin").write_bytes(payload)
    assert _run(exe, ["-k", "128", "-n", "160", "-e", "w.bin", "--matrix", "cauchy", "--threads", "4"],
                tmp_path).returncode == 0
    ff.write_conf(str(tmp_path / "c"), [f"_{r}_w.bin" for r in range(32, 160)])
    assert _run(exe, ["-d", "-i", "w.bin", "-c", "c", "-o", "o"], tmp_path).returncode == 0
    assert (tmp_path / "o").read_bytes() == payload
    (tmp_path / "w.bin.METADATA").write_text("12345\n32 128\n1 0 0\n")  # truncated matrix
    assert _run(exe, ["-d", "-i", "w.bin", "-c", "c", "-o", "o"], tmp_path).returncode == 1
    (tmp_path / "bad").write_text("_999_w.bin\n")
    assert _run(exe, ["-d", "-i", "w.bin", "-c", "bad"], tmp_path).returncode == 1


def test_asan_streaming_codec(exe, tmp_path):
    payload = os.urandom(250_007)
    (tmp_path / "s.bin").write_bytes(payload)
    assert _run(exe, ["-k", "10", "-n", "14", "-e", "s.bin", "--window", "4099", "--no-sync"], tmp_path).returncode == 0
    ff.write_conf(str(tmp_path / "c"), [f"_{r}_s.bin" for r in (0, 2, 3, 5, 6, 8, 10, 11, 12, 13)])
    assert _run(exe, ["-d", "-i", "s.bin", "-c", "c", "-o", "o", "--window", "1000", "--no-sync"],
                tmp_path).returncode == 0
    assert (tmp_path / "o").read_bytes() == payload


def test_asan_gf65536(exe, tmp_path):
    """GF(2^16) (-w 16): odd file size (even chunks, padded tail), a 340-chunk stripe past GF(2^8)'s
    n <= 256, the versioned METADATA, and a truncated version-2 matrix rejected."""
    payload = os.urandom(77_777)
    (tmp_path / "g.bin").write_bytes(payload)
    assert _run(exe, ["-k", "10", "-n", "14", "-w", "16", "-e", "g.bin"], tmp_path).returncode == 0
    assert (tmp_path / "g.bin.METADATA").read_text().startswith("GFRS-METADATA 2 16")
    ff.write_conf(str(tmp_path / "c"), [f"_{r}_g.bin" for r in (1, 2, 4, 5, 6, 7, 9, 10, 12, 13)])
    assert _run(exe, ["-d", "-i", "g.bin", "-c", "c", "-o", "o"], tmp_path).returncode == 0
    assert (tmp_path / "o").read_bytes() == payload

    wide = os.urandom(9_001)
    (tmp_path / "w.bin").write_bytes(wide)
    assert _run(exe, ["-k", "300", "-n", "340", "-w", "16", "-e", "w.bin", "--threads", "4"],
                tmp_path).returncode == 0
    ff.write_conf(str(tmp_path / "cw"), [f"_{r}_w.bin" for r in range(40, 340)])
    assert _run(exe, ["-d", "-i", "w.bin", "-c", "cw", "-o", "ow"], tmp_path).returncode == 0
    assert (tmp_path / "ow").read_bytes() == wide

    md = (tmp_path / "g.bin.METADATA").read_text().splitlines()
    (tmp_path / "g.bin.METADATA").write_text("\n".join(md[:4]) + "\n")  # header + part of the matrix
    assert _run(exe, ["-d", "-i", "g.bin", "-c", "c", "-o", "o2"], tmp_path).returncode == 1
