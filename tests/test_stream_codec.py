"""Bounded-memory, resumable file codec (csrc/io/stream_codec.cpp; SURVEY §5.4 checkpoint/resume).

The streamed encode must produce byte-identical chunk files and METADATA to the in-memory codec
(itself pinned to the reference cpu-rs.c by tests/test_cpu_codec.py), whatever the window size;
a run stopped after N windows (simulated crash) must resume from its checkpoint.
"""
import os
import subprocess
import sys

import pytest

from gpu_rscode_amd._build import binary
from gpu_rscode_amd._native import cpu
from gpu_rscode_amd.utils import fileformat as ff

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _files(d, name, n):
    return [(d / f"_{i}_{name}").read_bytes() for i in range(n)] + [(d / f"{name}.METADATA").read_bytes()]


def _encode_both(tmp_path, payload, k, p, window, matrix="vandermonde"):
    a, b = tmp_path / "mem", tmp_path / "str"
    a.mkdir()
    b.mkdir()
    (a / "f.bin").write_bytes(payload)
    (b / "f.bin").write_bytes(payload)
    cpu().encode_file(str(a / "f.bin"), k, p, matrix)
    r = cpu().encode_file_stream(str(b / "f.bin"), k, p, matrix, window=window, durable=False)
    return a, b, r


@pytest.mark.parametrize("size,k,p,window", [(3_000_017, 10, 4, 65536), (1 << 20, 4, 2, 4096),
                                             (12345, 16, 4, 100), (7, 4, 2, 1), (0, 3, 2, 0),
                                             (500_000, 128, 32, 1000)])
def test_stream_encode_equals_in_memory(tmp_path, size, k, p, window):
    payload = os.urandom(size)
    a, b, r = _encode_both(tmp_path, payload, k, p, window)
    assert r["complete"] and r["resumed_from"] == 0
    assert _files(a, "f.bin", k + p) == _files(b, "f.bin", k + p)
    assert not os.path.exists(str(b / "f.bin.PROGRESS"))


def test_stream_encode_resumes_after_crash(tmp_path):
    payload = os.urandom(2_000_003)
    d = tmp_path / "s"
    d.mkdir()
    f = str(d / "f.bin")
    (d / "f.bin").write_bytes(payload)
    W = 16384
    r1 = cpu().encode_file_stream(f, 10, 4, window=W, stop_after=5, durable=False)
    assert not r1["complete"] and r1["windows"] == 5
    assert os.path.exists(cpu().progress_path(f)) and not os.path.exists(f + ".METADATA")
    r2 = cpu().encode_file_stream(f, 10, 4, window=3 * W, durable=False)  # another window size is fine
    assert r2["complete"] and r2["resumed_from"] == 5 * W
    ref = tmp_path / "ref"
    ref.mkdir()
    (ref / "f.bin").write_bytes(payload)
    cpu().encode_file(str(ref / "f.bin"), 10, 4)
    assert _files(d, "f.bin", 14) == _files(ref, "f.bin", 14)


def test_stream_encode_checkpoint_for_other_parameters_is_ignored(tmp_path):
    payload = os.urandom(300_001)
    d = tmp_path / "s"
    d.mkdir()
    f = str(d / "f.bin")
    (d / "f.bin").write_bytes(payload)
    cpu().encode_file_stream(f, 10, 4, window=4096, stop_after=3, durable=False)
    r = cpu().encode_file_stream(f, 8, 4, window=4096, durable=False)  # different k: start over
    assert r["complete"] and r["resumed_from"] == 0
    r = cpu().encode_file_stream(f, 8, 4, window=4096, resume=False, durable=False)
    assert r["resumed_from"] == 0


def _conf(d, name, rows):
    conf = d / "conf"
    ff.write_conf(str(conf), [ff.chunk_path(str(d / name), r) for r in rows])
    return str(conf)


@pytest.mark.parametrize("rows", [(0, 2, 3, 5, 6, 8, 10, 11, 12, 13), (4, 5, 6, 7, 8, 9, 10, 11, 12, 13),
                                  tuple(range(10))])
def test_stream_decode_equals_payload(tmp_path, rows):
    payload = os.urandom(1_000_003)
    d = tmp_path / "s"
    d.mkdir()
    f = str(d / "f.bin")
    (d / "f.bin").write_bytes(payload)
    cpu().encode_file_stream(f, 10, 4, window=8192, durable=False)
    r = cpu().decode_file_stream(f, _conf(d, "f.bin", rows), str(d / "out"), window=10000, durable=False)
    assert r["complete"] and r["erased"] == sum(1 for x in range(10) if x not in rows)
    assert (d / "out").read_bytes() == payload


def test_stream_decode_resume_and_corruption(tmp_path):
    payload = os.urandom(777_777)
    d = tmp_path / "s"
    d.mkdir()
    f = str(d / "f.bin")
    (d / "f.bin").write_bytes(payload)
    cpu().encode_file(f, 10, 4)
    bad = d / "_3_f.bin"
    raw = bytearray(bad.read_bytes())
    raw[12345] ^= 0x40
    bad.write_bytes(bytes(raw))  # CRC mismatch: skipped, a spare from the conf is used instead
    conf = _conf(d, "f.bin", (0, 1, 3, 4, 5, 6, 7, 8, 9, 10, 12))
    out = str(d / "out")
    r1 = cpu().decode_file_stream(f, conf, out, window=4096, stop_after=4, durable=False)
    assert not r1["complete"] and r1["rejected"] == 1
    r2 = cpu().decode_file_stream(f, conf, out, window=4096, durable=False)
    assert r2["complete"] and r2["resumed_from"] == 4 * 4096
    assert (d / "out").read_bytes() == payload


def test_cpu_rs_cli_streaming_flags(tmp_path):
    exe = str(binary("CPU-RS"))
    payload = os.urandom(654_321)
    (tmp_path / "f.bin").write_bytes(payload)
    subprocess.run([exe, "-k", "6", "-n", "9", "-e", "f.bin", "--window", "32768", "--no-sync"], cwd=tmp_path,
                   check=True, capture_output=True, timeout=120)
    subprocess.run([exe, "-k", "6", "-n", "9", "-e", "f.bin", "--make-conf"], cwd=tmp_path, check=True,
                   capture_output=True, timeout=60)
    r = subprocess.run([exe, "-d", "-i", "f.bin", "-c", "conf-9-6-f.bin", "-o", "out.bin", "--window", "0"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "out.bin").read_bytes() == payload


def test_python_cli_streaming_cpu_backend(tmp_path):
    from gpu_rscode_amd.utils.cli import main
    payload = os.urandom(100_003)
    f = tmp_path / "f.bin"
    f.write_bytes(payload)
    assert main(["-k", "5", "-n", "8", "-e", str(f), "--backend", "cpu", "--window", "777", "--no-sync", "-q"]) == 0
    conf = tmp_path / "conf"
    ff.write_conf(str(conf), [ff.chunk_path(str(f), r) for r in (1, 2, 5, 6, 7)])
    assert main(["-d", "-i", str(f), "-c", str(conf), "-o", str(tmp_path / "o"), "--backend", "cpu",
                 "--window", "0", "-q"]) == 0
    assert (tmp_path / "o").read_bytes() == payload


def test_crc32_combine_matches_zlib():
    import zlib

    rng = os.urandom
    for la, lb in [(0, 0), (1, 0), (0, 5), (1, 1), (17, 4095), (100_003, 65_537), (3, 1 << 20)]:
        a, b = rng(la), rng(lb)
        assert cpu().crc32(a) == zlib.crc32(a)
        assert cpu().crc32_combine(cpu().crc32(a), cpu().crc32(b), lb) == zlib.crc32(a + b)


def test_crc32_fast_path_matches_zlib_and_the_table_path():
    """The carry-less-multiply CRC-32 (64-byte folds, then 16-byte folds, then the table for the
    tail) equals zlib for every length around its block sizes, unaligned starts and chained seeds;
    the slicing-by-8 table path (GFRS_TUNE=crc=scalar, a fresh process) gives the same values."""
    import zlib

    buf = os.urandom(1 << 18)
    cases = [(n, off, seed) for n in list(range(0, 200)) + [1023, 1024, 1025, 4096 + 15, 65_599, 200_000]
             for off, seed in ((0, 0), (3, 0x12345678), (13, 0xFFFFFFFF))]
    want = [zlib.crc32(buf[off:off + n], seed) for n, off, seed in cases]
    assert [cpu().crc32(buf[off:off + n], seed) for n, off, seed in cases] == want
    code = ("import sys, zlib, os; sys.path.insert(0, sys.argv[1]); from gpu_rscode_amd._native import cpu; "
            "b = os.urandom(70_001); assert cpu().crc32(b, 7) == zlib.crc32(b, 7); print('ok')")
    r = subprocess.run([sys.executable, "-c", code, ROOT], env=dict(os.environ, GFRS_TUNE="crc=scalar"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def test_stream_decode_skips_corrupt_and_missing_survivors(tmp_path):
    """The windowed decoder's survivor check (the first k candidates read and CRC-checked at once):
    a corrupted chunk and a missing chunk among the first k are skipped, the next listed chunks take
    their place, and the file comes back byte-exact."""
    f = tmp_path / "f.bin"
    payload = os.urandom(500_001)
    f.write_bytes(payload)
    cpu().encode_file(str(f), 6, 3)
    bad = bytearray((tmp_path / "_2_f.bin").read_bytes())
    bad[7] ^= 0x40
    (tmp_path / "_2_f.bin").write_bytes(bytes(bad))
    os.remove(tmp_path / "_4_f.bin")
    ff.write_conf(str(tmp_path / "conf"), [ff.chunk_path(str(f), i) for i in range(9)])
    rows, rejected = cpu().choose_survivors(str(f), str(tmp_path / "conf"))
    assert rejected == 1 and rows == [0, 1, 3, 5, 6, 7]
    r = cpu().decode_file_stream(str(f), str(tmp_path / "conf"), str(tmp_path / "o"), window=70_000, durable=False)
    assert r["rejected"] == 1 and (tmp_path / "o").read_bytes() == payload


@pytest.mark.parametrize("size,k,p,w,cuts", [(3_000_017, 10, 4, 8, (0, 100_000, 222_224, None)),
                                             (1_000_001, 10, 4, 16, (0, 4096, 50_002, None)),
                                             (99_999, 6, 3, 8, (0, 0, 16_667, None))])
def test_column_shards_equal_the_whole_encode(tmp_path, size, k, p, w, cuts):
    """The multi-GPU file codec's building block: every shard [lo, hi) of the columns encoded on its
    own into pre-sized chunk files (shard=True: no truncation, no METADATA, per-shard checkpoint),
    shard CRCs combined in column order == the one-call encode's files and METADATA CRCs (an empty
    shard included)."""
    payload = os.urandom(size)
    ref, sh = tmp_path / "ref", tmp_path / "sh"
    ref.mkdir()
    sh.mkdir()
    (ref / "f.bin").write_bytes(payload)
    (sh / "f.bin").write_bytes(payload)
    cpu().encode_file_stream(str(ref / "f.bin"), k, p, window=8192, durable=False, field_w=w)
    C = ff.chunk_size(size, k, w)
    for i in range(k + p):
        with open(ff.chunk_path(str(sh / "f.bin"), i), "wb") as fh:
            fh.truncate(C)
    bounds = [c if c is not None else C for c in cuts]
    crc = [0] * (k + p)
    for lo, hi in zip(bounds, bounds[1:]):
        r = cpu().encode_file_stream(str(sh / "f.bin"), k, p, window=6000, durable=False, field_w=w, col_lo=lo,
                                     col_hi=hi, shard=True)
        assert r["complete"] and (r["col_lo"], r["col_hi"]) == (lo, hi) and len(r["crc"]) == k + p
        crc = [cpu().crc32_combine(a, b, hi - lo) for a, b in zip(crc, r["crc"])]
        assert not os.path.exists(str(sh / "f.bin.METADATA"))
    md = ff.read_metadata(str(ref / "f.bin.METADATA"))
    assert crc == md.crc
    for i in range(k + p):
        assert (sh / f"_{i}_f.bin").read_bytes() == (ref / f"_{i}_f.bin").read_bytes(), i
    # shard decode with a coordinator-chosen survivor list, each shard into the pre-sized output
    rows, rejected = cpu().choose_survivors(str(ref / "f.bin"), _conf(ref, "f.bin", list(range(p, k + p))))
    assert rejected == 0 and rows == list(range(p, k + p))
    out = tmp_path / "out"
    with open(out, "wb") as fh:
        fh.truncate(size)
    for lo, hi in zip(bounds, bounds[1:]):
        r = cpu().decode_file_stream(str(ref / "f.bin"), str(ref / "conf"), str(out), window=5000, durable=False,
                                     col_lo=lo, col_hi=hi, shard=True, rows=rows)
        assert r["complete"] and r["rows"] == rows
    assert out.read_bytes() == payload


def test_stream_w16_roundtrip_with_resume(tmp_path):
    """GF(2^16) through the windowed codec: a crash after 3 windows, resume, files identical to the
    in-memory GF(2^16) encode; the streamed decode (another crash + resume) restores the payload."""
    payload = os.urandom(1_234_567)
    a, b = tmp_path / "mem", tmp_path / "str"
    a.mkdir()
    b.mkdir()
    (a / "f.bin").write_bytes(payload)
    (b / "f.bin").write_bytes(payload)
    cpu().encode_file(str(a / "f.bin"), 10, 4, field_w=16)
    f = str(b / "f.bin")
    r1 = cpu().encode_file_stream(f, 10, 4, window=8191, stop_after=3, durable=False, field_w=16)
    assert not r1["complete"] and r1["window"] % 2 == 0
    r2 = cpu().encode_file_stream(f, 10, 4, window=8191, durable=False, field_w=16)
    assert r2["complete"] and r2["resumed_from"] == 3 * r1["window"]
    assert _files(a, "f.bin", 14) == _files(b, "f.bin", 14)
    conf = _conf(b, "f.bin", (4, 5, 6, 7, 8, 9, 10, 11, 12, 13))
    out = str(b / "out")
    r3 = cpu().decode_file_stream(f, conf, out, window=4097, stop_after=2, durable=False)
    assert not r3["complete"]
    r4 = cpu().decode_file_stream(f, conf, out, window=4097, durable=False)
    assert r4["complete"] and r4["resumed_from"] > 0 and r4["erased"] == 4
    assert (b / "out").read_bytes() == payload


def test_cpu_rs_cli_w16_window(tmp_path):
    exe = str(binary("CPU-RS"))
    payload = os.urandom(300_001)
    (tmp_path / "f.bin").write_bytes(payload)
    r = subprocess.run([exe, "-k", "300", "-n", "340", "-w", "16", "-e", "f.bin", "--window", "512", "--no-sync", "-q"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    md = ff.read_metadata(str(tmp_path / "f.bin.METADATA"))
    assert md.w == 16 and md.k == 300
    ff.write_conf(str(tmp_path / "conf"), ff.worst_case_conf("f.bin", 340, 300))
    r = subprocess.run([exe, "-d", "-i", "f.bin", "-c", "conf", "-o", "o.bin", "--window", "0", "-q"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "o.bin").read_bytes() == payload
