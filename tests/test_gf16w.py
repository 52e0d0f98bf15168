"""GF(2^16) — the w = 16 member of the reference's field family (src/galoisfield.cu:22-32, poly
0210013 = 0x1100B; never built there). Host side: the C++ field (csrc/include/gfrs/gf65536.h)
against the numpy oracle, the four-byte-map decomposition the gfx950 kernel applies, the C++ CPU
GEMM, the ReedSolomon codec, the versioned METADATA and the CLIs (-w 16)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from gpu_rscode_amd import ReedSolomon, UnrecoverableError, gf
from gpu_rscode_amd._native import cpu
from gpu_rscode_amd.utils import fileformat as ff

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
F = gf.field(16)


def test_field_is_the_reference_polynomial():
    assert F.poly == 0o210013 == 0x1100B
    # generator 2 has order 65535 (primitive): every nonzero element has a log
    assert np.all(F.log[1:] >= 0) and F.exp[65534] != 1 and F.mul(F.exp[65534], 2) == 1


def test_cpp_field_matches_oracle():
    rng = np.random.default_rng(0)
    a, b = rng.integers(0, 65536, 2000), rng.integers(0, 65536, 2000)
    want = F.mul(a, b)
    got = [cpu().gf16_mul(int(x), int(y)) for x, y in zip(a, b)]
    assert np.array_equal(np.array(got), want)
    m = rng.integers(0, 65536, size=(12, 12))
    inv = np.array(cpu().gf16_invert([int(v) for v in m.reshape(-1)], 12)).reshape(12, 12)
    assert np.array_equal(inv, F.invert(m))
    assert np.array_equal(F.matmul(m, inv), np.eye(12, dtype=np.uint16))
    with pytest.raises(ValueError):
        cpu().gf16_invert([1, 2, 2, 4], 2)  # rows dependent: singular


def test_four_byte_maps_reproduce_the_multiply():
    """c * (l | h<<8) = [L_ll(l) ^ L_hl(h)] | [L_lh(l) ^ L_hh(h)] << 8, each map one v_perm record;
    the numpy and C++ records are the same words."""
    rng = np.random.default_rng(1)
    c = rng.integers(0, 65536, size=(4, 6))
    c[0, 0], c[0, 1], c[1, 0] = 0, 1, 65535
    quads = gf.perm_quads16(c)
    x = np.arange(65536, dtype=np.uint16)
    for i in range(4):
        for j in range(6):
            assert np.array_equal(gf.quad_apply16(quads[i, j], x), F.mul(int(c[i, j]), x).astype(np.uint16))
            assert list(quads[i, j].reshape(-1)) == cpu().gf16_perm_quad(int(c[i, j]))


@pytest.mark.parametrize("k,n", [(10, 14), (300, 340)])
def test_codec_cpu_roundtrip_beyond_256_chunks(k, n):
    rs = ReedSolomon(k, n, field="gf65536")
    assert rs.G.dtype == np.uint16 and rs.G.shape == (n, k)
    rng = np.random.default_rng(k)
    C = 2 * 501
    data = torch.from_numpy(rng.integers(0, 256, size=(k, C), dtype=np.uint8))
    par = rs.encode(data)
    assert np.array_equal(par.numpy().view("<u2"), F.gemm(rs.E, data.numpy().view("<u2")))
    stripe = torch.cat([data, par])
    erased = sorted(rng.choice(k, size=n - k, replace=False).tolist())  # only natives: always recoverable
    rows = [r for r in range(n) if r not in erased]
    assert torch.equal(rs.decode(stripe[rows], rows), data)


def test_mds_matrices_and_singular_patterns():
    k, n = 6, 10
    for kind in ("cauchy", "sys_vandermonde"):
        rs = ReedSolomon(k, n, matrix=kind, field="gf65536")
        if kind == "cauchy":
            want = F.inv(np.arange(k, n)[:, None] ^ np.arange(k)[None, :])
            assert np.array_equal(rs.E, want)
        assert not F.singular_patterns(rs.G, k)  # every k-subset invertible
    rs = ReedSolomon(2, 4, field="gf65536")
    rs.G = np.array([[1, 0], [0, 1], [1, 1], [1, 1]], dtype=np.uint16)  # rows 2 and 3 equal
    with pytest.raises(UnrecoverableError):
        rs.decode_matrix([2, 3])


@pytest.mark.parametrize("matrix", ["vandermonde", "cauchy"])
def test_erased_rows_solve_matches_the_full_inverse(matrix):
    """The e x e systematic solve (gf16_decode_rows) gives exactly the erased rows of the full
    inverse, for random patterns, survivors in any order, and wanted rows that survived."""
    k, n = 24, 34
    rs = ReedSolomon(k, n, matrix=matrix, field="gf65536")
    g = np.random.default_rng(5)
    for _ in range(25):
        rows = [int(r) for r in g.permutation(n)[:k]]
        if not rs.is_recoverable(rows):
            with pytest.raises(UnrecoverableError):
                rs._erased_rows(rows, [i for i in range(k) if i not in rows])
            continue
        full = rs.decode_matrix(rows)
        erased = [i for i in range(k) if i not in rows]
        assert np.array_equal(rs._erased_rows(rows, erased), full[erased])
        some = [0, k - 1, erased[0]] if erased else [0]
        raw = cpu().gf16_decode_rows(np.ascontiguousarray(rs.G, dtype="<u2").tobytes(), k, rows, some)
        assert np.array_equal(np.frombuffer(raw, dtype="<u2").reshape(len(some), k), full[some])
    g2 = np.array(rs.G)  # a non-systematic G takes the full-inverse fallback
    g2[0, 1] ^= 1
    rs.G = g2  # (assigning G drops the patterns cached for the old one)
    rows = list(range(n - k, n))
    a = rs.G[rows]
    inv = np.asarray(cpu().gf16_invert([int(v) for v in a.reshape(-1)], k), dtype=np.uint16).reshape(k, k)
    erased = list(range(n - k))
    assert np.array_equal(rs._erased_rows(rows, erased), inv[erased])
    rs2 = ReedSolomon(2, 4, field="gf65536")
    rs2.G = np.array([[1, 0], [0, 1], [1, 1], [1, 1]], dtype=np.uint16)  # rows 2 and 3 equal: singular
    with pytest.raises(UnrecoverableError):
        rs2._erased_rows([2, 3], [0, 1])


def test_bad_inputs_are_rejected():
    """Wanted rows are range-checked on both paths (the full-inverse fallback included), chunk ids
    against n, and gf16_invert's entry count against n * n."""
    k, n = 6, 9
    rs = ReedSolomon(k, n, field="gf65536")
    gb = np.ascontiguousarray(rs.G, dtype="<u2").tobytes()
    rows = list(range(n - k, n))
    g2 = np.array(rs.G)
    g2[0, 1] ^= 1  # non-systematic: the fallback path
    for gbytes in (gb, np.ascontiguousarray(g2, dtype="<u2").tobytes()):
        for bad in ([-1], [k], [0, 10_000]):
            with pytest.raises(ValueError):
                cpu().gf16_decode_rows(gbytes, k, rows, bad)
    with pytest.raises(ValueError):
        cpu().gf16_decode_rows(gb, k, [0, 1, 2, 3, 4, n], [0])
    with pytest.raises(ValueError):
        cpu().gf16_invert([1, 0, 0], 2)
    with pytest.raises(ValueError):
        cpu().gf16_invert([1, 0, 0, 1], 3)
    with pytest.raises(ValueError):
        cpu().gf16_invert([1, 0, 0, 70000], 2)


def test_odd_byte_rows_are_rejected():
    rs = ReedSolomon(4, 6, field="gf65536")
    with pytest.raises(ValueError, match="even byte count"):
        rs.encode(torch.zeros((4, 101), dtype=torch.uint8))


def test_versioned_metadata_roundtrip(tmp_path):
    e = F.vandermonde_ref(300, 40)
    p = str(tmp_path / "x.METADATA")
    ff.write_metadata(p, 12345, 40, 300, e, crc=list(range(340)), w=16)
    assert open(p).readline() == "GFRS-METADATA 2 16\n"
    md = ff.read_metadata(p)
    assert md.w == 16 and md.k == 300 and md.p == 40 and md.g.dtype == np.uint16
    assert np.array_equal(md.e, e) and md.crc == list(range(340))
    d = cpu().read_metadata(p)  # the C++ reader agrees
    assert d["w"] == 16 and np.array_equal(np.array(d["g"]).reshape(340, 300)[300:], e)
    with open(p, "w") as f:
        f.write("GFRS-METADATA 3 16\n1\n1 1\n")
    with pytest.raises(ValueError):
        ff.read_metadata(p)
    with pytest.raises(RuntimeError):
        cpu().read_metadata(p)


def _cpu_rs(args, cwd):
    return subprocess.run([os.path.join(ROOT, "bin", "CPU-RS"), *args], cwd=cwd, capture_output=True, text=True,
                          timeout=300)


@pytest.mark.parametrize("k,n,size", [(10, 14, 1_000_001), (300, 340, 300_007)])
def test_cpu_cli_w16_roundtrip(tmp_path, k, n, size):
    payload = np.random.default_rng(size).integers(0, 256, size, dtype=np.uint8).tobytes()
    (tmp_path / "f.bin").write_bytes(payload)
    r = _cpu_rs(["-q", "-k", str(k), "-n", str(n), "-w", "16", "-e", "f.bin"], tmp_path)
    assert r.returncode == 0, r.stderr
    md = ff.read_metadata(str(tmp_path / "f.bin.METADATA"))
    C = ff.chunk_size(size, k, 16)
    assert md.w == 16 and C % 2 == 0 and (tmp_path / "_0_f.bin").stat().st_size == C
    # parity is the oracle's, over little-endian 16-bit symbols of the zero-padded stripe
    data = np.frombuffer(payload + bytes(k * C - size), dtype=np.uint8).reshape(k, C)
    par = np.stack([np.frombuffer((tmp_path / f"_{k + i}_f.bin").read_bytes(), dtype=np.uint8) for i in range(n - k)])
    assert np.array_equal(par.view("<u2")[:, :64], F.gemm(md.e, data.view("<u2")[:, :64]))
    # lose n - k natives (the reference's unit-test.sh pattern), decode from the rest
    ff.write_conf(str(tmp_path / "conf"), ff.worst_case_conf("f.bin", n, k))
    r = _cpu_rs(["-q", "-d", "-i", "f.bin", "-c", "conf", "-o", "o.bin"], tmp_path)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "o.bin").read_bytes() == payload


def test_cli_field_width_validation(tmp_path):
    (tmp_path / "f.bin").write_bytes(b"x" * 100)
    assert _cpu_rs(["-k", "300", "-n", "340", "-e", "f.bin"], tmp_path).returncode == 2  # n > 256 needs -w 16
    assert _cpu_rs(["-k", "4", "-n", "6", "-w", "12", "-e", "f.bin"], tmp_path).returncode == 2
    assert _cpu_rs(["-k", "4", "-n", "6", "-w", "16", "--cpu-meta", "-e", "f.bin"], tmp_path).returncode == 2


def test_python_cli_w16(tmp_path):
    payload = os.urandom(77_777)
    (tmp_path / "f.bin").write_bytes(payload)
    env = dict(os.environ, PYTHONPATH=ROOT)
    py = [sys.executable, "-m", "gpu_rscode_amd"]
    r = subprocess.run(py + ["-k", "5", "-n", "8", "-w", "16", "-e", "f.bin", "--backend", "cpu"], cwd=tmp_path,
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr
    ff.write_conf(str(tmp_path / "conf"), [f"_{i}_f.bin" for i in (1, 3, 5, 6, 7)])
    r = subprocess.run(py + ["-d", "-i", "f.bin", "-c", "conf", "-o", "o.bin", "--backend", "cpu"], cwd=tmp_path,
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "o.bin").read_bytes() == payload
