"""C++ CPU reference codec, descriptors, file formats and CLIs (CPU only).

Parity fixture: tests/fixtures/golden_parity.json holds SHA-256 digests of the chunk files the
reference's own CPU codec (src/cpu-rs.c, compiled with gcc in /tmp — never in this repo) wrote
for deterministic inputs; our encoder must reproduce them bit for bit (BASELINE config #1).
"""
import hashlib
import itertools
import json
import os
import subprocess

import numpy as np
import pytest
import torch

from gpu_rscode_amd import ReedSolomon, gf
from gpu_rscode_amd.gf import GF256
from gpu_rscode_amd._native import cpu
from gpu_rscode_amd._build import binary
from gpu_rscode_amd.ops.gemm import build_desc, desc_layout, pad_m, perm_tables_from_coeff
from gpu_rscode_amd.utils import fileformat as ff

FIX = os.path.join(os.path.dirname(__file__), "fixtures", "golden_parity.json")
STRATEGIES = ["logexp", "logexp0", "logexp1", "logexp2", "logexp3", "loop", "full", "double", "perm", "row", "simd"]


def golden_input(n: int) -> bytes:
    out = bytearray()
    i = 0
    while len(out) < n:
        out += hashlib.sha256(b"gpu_rscode_amd-golden" + i.to_bytes(8, "little")).digest()
        i += 1
    return bytes(out[:n])


def sha(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


# ---- descriptors -------------------------------------------------------------------------------
@pytest.mark.parametrize("k,m,batch", [(1, 1, 1), (4, 2, 1), (10, 4, 1), (10, 3, 7), (16, 4, 1), (128, 32, 1),
                                       (7, 17, 3), (255, 1, 1), (10, 4, 1000)])
def test_desc_layout_python_equals_native(k, m, batch):
    mp = pad_m(m)
    assert cpu().pad_m(m) == mp
    lay = desc_layout(k, mp, batch)
    nat = cpu().desc_layout(k, mp, batch)
    assert (lay.in_off, lay.copy_off, lay.out_off, lay.tab_off, lay.bytes) == (
        nat["in_off"], nat["copy_off"], nat["out_off"], nat["tab_off"], nat["bytes"])


@pytest.mark.parametrize("k,m,batch", [(10, 4, 1), (300, 40, 1), (300, 40, 256), (7, 3, 5), (64, 16, 9)])
def test_desc_layout16_python_equals_native(k, m, batch):
    from gpu_rscode_amd.ops.gemm import desc_layout16

    mp = pad_m(m)
    lay = desc_layout16(k, mp, batch)
    nat = cpu().desc_layout16(k, mp, batch)
    assert (lay.in_off, lay.copy_off, lay.out_off, lay.tab_off, lay.bytes) == (
        nat["in_off"], nat["copy_off"], nat["out_off"], nat["tab_off"], nat["bytes"])


def test_build_desc_python_equals_native():
    k, m = 10, 3
    coeff = np.random.default_rng(0).integers(0, 256, size=(m, k), dtype=np.uint8)
    ins = [0x1000 * (j + 1) for j in range(k)]
    outs = [0x900000 + 0x100 * i for i in range(m)]
    copies = [0x77770000 + j if j % 3 == 0 else 0 for j in range(k)]
    py = build_desc(ins, outs, copies, perm_tables_from_coeff(coeff))
    nat = np.frombuffer(cpu().build_desc(k, m, ins, copies, outs, coeff.tobytes()), dtype=np.uint8)
    assert np.array_equal(py, nat)


# ---- multiply strategies (the reference's nine CPU programs) -----------------------------------
@pytest.mark.parametrize("strategy", STRATEGIES)
def test_every_strategy_matches_oracle(strategy):
    rng = np.random.default_rng(hash(strategy) % 2**32)
    for a, b in rng.integers(0, 256, size=(400, 2)).tolist() + [(0, 0), (0, 7), (7, 0), (255, 255), (1, 1)]:
        assert cpu().mul_strategy(strategy, a, b) == int(GF256.mul(a, b)), (strategy, a, b)


@pytest.mark.parametrize("strategy", STRATEGIES)
@pytest.mark.parametrize("k,m,ncols", [(4, 2, 1000), (10, 4, 4099), (3, 3, 1), (7, 9, 16447), (1, 6, 33)])
def test_cpu_gemm_matches_oracle(strategy, k, m, ncols):
    rng = np.random.default_rng(k * m + ncols)
    coeff = rng.integers(0, 256, size=(m, k), dtype=np.uint8)
    data = rng.integers(0, 256, size=(k, ncols), dtype=np.uint8)
    out = np.zeros((m, ncols), dtype=np.uint8)
    cpu().gemm([data[j].ctypes.data for j in range(k)], [out[i].ctypes.data for i in range(m)], coeff.tobytes(),
               ncols, strategy, 1)
    assert np.array_equal(out, GF256.gemm(coeff, data))


@pytest.mark.parametrize("strategy,m", [("row", 4), ("simd", 4), ("simd", 6)])
def test_cpu_gemm_multithreaded(strategy, m):
    k, ncols = 10, (3 << 20) + 13
    rng = np.random.default_rng(5)
    coeff = rng.integers(0, 256, size=(m, k), dtype=np.uint8)
    data = rng.integers(0, 256, size=(k, ncols), dtype=np.uint8)
    out = np.zeros((m, ncols), dtype=np.uint8)
    cpu().gemm([data[j].ctypes.data for j in range(k)], [out[i].ctypes.data for i in range(m)], coeff.tobytes(),
               ncols, strategy, 4)
    assert np.array_equal(out, GF256.gemm(coeff, data))


# ---- host matrix algebra -----------------------------------------------------------------------
@pytest.mark.parametrize("kind", ["vandermonde", "cauchy", "sys_vandermonde"])
def test_native_encoding_matrix_equals_oracle(kind):
    for k, p in [(4, 2), (10, 4), (16, 4), (128, 32)]:
        nat = np.frombuffer(cpu().encoding_matrix(kind, k, p), dtype=np.uint8).reshape(p, k)
        assert np.array_equal(nat, GF256.encoding_matrix(kind, k, p)), (kind, k, p)


def test_native_invert_and_singular():
    g = GF256.generator(GF256.vandermonde_ref(10, 4))
    for rows in [(0, 1, 2, 3, 4, 5, 6, 10, 11, 12), (4, 5, 6, 7, 8, 9, 10, 11, 12, 13)]:
        nat = np.frombuffer(cpu().decode_matrix(g.tobytes(), 10, list(rows)), dtype=np.uint8).reshape(10, 10)
        assert np.array_equal(nat, GF256.invert(g[list(rows)]))
    for bad in GF256.singular_patterns(g, 10):
        assert cpu().decode_matrix(g.tobytes(), 10, list(bad)) is None


# ---- model on CPU tensors ----------------------------------------------------------------------
@pytest.mark.parametrize("matrix", ["vandermonde", "cauchy"])
def test_reed_solomon_cpu_all_erasure_subsets_k4_n6(matrix):
    k, n = 4, 6
    rs = ReedSolomon(k, n, matrix=matrix)
    data = torch.from_numpy(np.random.default_rng(1).integers(0, 256, size=(k, 3001), dtype=np.uint8))
    parity = rs.encode(data)
    assert np.array_equal(parity.numpy(), GF256.gemm(rs.E, data.numpy()))
    stripe = [data[i] for i in range(k)] + [parity[i] for i in range(n - k)]
    for rows in itertools.combinations(range(n), k):
        out = rs.decode([stripe[r].clone() for r in rows], rows)
        assert torch.equal(out, data), rows


def test_reed_solomon_cpu_reconstruct_mixed():
    k, n = 10, 14
    rs = ReedSolomon(k, n)
    data = torch.from_numpy(np.random.default_rng(2).integers(0, 256, size=(k, 999), dtype=np.uint8))
    parity = rs.encode(data)
    full = torch.cat([data, parity])
    broken = full.clone()
    erased = [1, 7, 11, 13]
    broken[erased] = 0
    rs.reconstruct(broken, erased)
    assert torch.equal(broken, full)


def test_reed_solomon_unrecoverable_pattern_raises():
    from gpu_rscode_amd import UnrecoverableError

    rs = ReedSolomon(10, 14)
    bad = GF256.singular_patterns(rs.G, 10)[0]
    assert not rs.is_recoverable(bad)
    with pytest.raises(UnrecoverableError):
        rs.decode_matrix(bad)


def test_reed_solomon_gf16_cpu_roundtrip():
    rs = ReedSolomon(4, 6, field="gf16")
    data = torch.from_numpy(np.random.default_rng(3).integers(0, 256, size=(4, 777), dtype=np.uint8))
    parity = rs.encode(data)
    stripe = [data[i] for i in range(4)] + [parity[i] for i in range(2)]
    for rows in itertools.combinations(range(6), 4):
        assert torch.equal(rs.decode([stripe[r] for r in rows], rows), data)


# ---- file formats ------------------------------------------------------------------------------
def test_chunk_names_and_index():
    assert ff.chunk_path("f.bin", 3) == "_3_f.bin" == cpu().chunk_path("f.bin", 3)
    assert ff.chunk_path("a/b/f.bin", 12) == "a/b/_12_f.bin" == cpu().chunk_path("a/b/f.bin", 12)
    assert ff.chunk_index("_12_f.bin") == 12 == cpu().chunk_index("x/_12_f.bin")
    assert ff.chunk_index("f.bin") == -1 == cpu().chunk_index("f.bin")


def test_metadata_roundtrip_both_formats(tmp_path):
    e = GF256.vandermonde_ref(4, 2)
    p = str(tmp_path / "m.METADATA")
    ff.write_metadata(p, 12345, 2, 4, e)
    md = ff.read_metadata(p)
    assert md.has_matrix and md.total_size == 12345 and np.array_equal(md.e, e)
    nat = cpu().read_metadata(p)
    assert nat["has_matrix"] and np.array_equal(np.frombuffer(nat["g"], np.uint8).reshape(6, 4), md.g)
    text = open(p).read().splitlines()
    assert text[:3] == ["12345", "2 4", "1 0 0 0 "]  # reference write_metadata layout
    ff.write_metadata(p, 99, 2, 4, None, with_matrix=False)  # cpu-rs.c 2-line form
    md = ff.read_metadata(p)
    assert not md.has_matrix and np.array_equal(md.e, e)


def test_worst_case_conf_matches_unit_test_sh():
    assert ff.worst_case_conf("f", 6, 4) == ["_2_f", "_3_f", "_4_f", "_5_f"]
    assert cpu().worst_case_conf("f", 6, 4) == ff.worst_case_conf("f", 6, 4)


# ---- file-level codec --------------------------------------------------------------------------
@pytest.mark.parametrize("case", ["4,6,1000003", "10,14,1000003", "8,11,65536"])
def test_golden_parity_equals_reference_cpu_rs(tmp_path, case):
    k, n, size = map(int, case.split(","))
    golden = json.load(open(FIX))["cases"][case]
    f = tmp_path / "in.bin"
    f.write_bytes(golden_input(size))
    cpu().encode_file(str(f), k, n - k)
    for i in range(n):
        assert sha(tmp_path / f"_{i}_in.bin") == golden[str(i)], f"chunk {i}"


def test_file_roundtrip_every_erasure_subset_k4_n6(tmp_path):
    k, n = 4, 6
    f = tmp_path / "f.bin"
    payload = os.urandom(100_003)
    f.write_bytes(payload)
    cpu().encode_file(str(f), k, n - k)
    for rows in itertools.combinations(range(n), k):
        conf = tmp_path / "conf"
        ff.write_conf(str(conf), [ff.chunk_path(str(f), r) for r in rows])
        out = tmp_path / "out.bin"
        cpu().decode_file(str(f), str(conf), str(out))
        assert out.read_bytes() == payload, rows


def test_file_decode_singular_pattern_errors(tmp_path):
    f = tmp_path / "f.bin"
    f.write_bytes(os.urandom(5000))
    cpu().encode_file(str(f), 10, 4)
    g = GF256.generator(GF256.vandermonde_ref(10, 4))
    bad = GF256.singular_patterns(g, 10)[0]
    conf = tmp_path / "conf"
    ff.write_conf(str(conf), [ff.chunk_path(str(f), r) for r in bad])
    with pytest.raises(RuntimeError, match="unrecoverable"):
        cpu().decode_file(str(f), str(conf), str(tmp_path / "o"))


def test_file_decode_accepts_cpu_metadata(tmp_path):
    f = tmp_path / "f.bin"
    payload = os.urandom(7777)
    f.write_bytes(payload)
    cpu().encode_file(str(f), 4, 2, cpu_meta=True)
    assert len(open(str(f) + ".METADATA").read().split()) == 3
    conf = tmp_path / "c"
    ff.write_conf(str(conf), ff.worst_case_conf(str(f), 6, 4))
    cpu().decode_file(str(f), str(conf), str(tmp_path / "o"))
    assert (tmp_path / "o").read_bytes() == payload


# ---- CLI ---------------------------------------------------------------------------------------
def run(cmd, cwd):
    return subprocess.run(cmd, cwd=cwd, capture_output=True, text=True, timeout=120)


def test_cpu_rs_cli_roundtrip_reference_flags(tmp_path):
    exe = str(binary("CPU-RS"))
    payload = os.urandom(1 << 20)
    (tmp_path / "f.bin").write_bytes(payload)
    r = run([exe, "-K", "4", "-N", "6", "-E", "f.bin"], tmp_path)  # uppercase aliases take arguments
    assert r.returncode == 0, r.stderr
    r = run([exe, "-k", "4", "-n", "6", "-e", "f.bin", "--make-conf"], tmp_path)
    assert r.returncode == 0 and (tmp_path / "conf-6-4-f.bin").exists()
    r = run([exe, "-d", "-i", "f.bin", "-c", "conf-6-4-f.bin", "-o", "out.bin"], tmp_path)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "out.bin").read_bytes() == payload
    # without -o the decoder overwrites the input file (reference behaviour, src/decode.cu:410-425)
    (tmp_path / "f.bin").write_bytes(b"garbage")
    r = run([exe, "-d", "-i", "f.bin", "-c", "conf-6-4-f.bin"], tmp_path)
    assert r.returncode == 0 and (tmp_path / "f.bin").read_bytes() == payload


def test_cpu_rs_cli_validation(tmp_path):
    exe = str(binary("CPU-RS"))
    assert run([exe, "-h"], tmp_path).returncode == 0
    assert run([exe], tmp_path).returncode != 0
    assert run([exe, "-k", "0", "-n", "4", "-e", "x"], tmp_path).returncode != 0
    assert run([exe, "-d", "-i", "x"], tmp_path).returncode != 0
    assert run([exe, "-k", "4", "-n", "6", "-e", "missing.bin"], tmp_path).returncode == 1


# ---- failure detection: checksums and aggressive read -----------------------------------------
def test_metadata_crc_extension_and_corruption_detection(tmp_path):
    import zlib

    f = tmp_path / "f.bin"
    payload = os.urandom(60_001)
    f.write_bytes(payload)
    cpu().encode_file(str(f), 4, 3)
    md = ff.read_metadata(str(f) + ".METADATA")
    assert md.crc is not None and len(md.crc) == 7
    for i in range(7):
        assert md.crc[i] == zlib.crc32((tmp_path / f"_{i}_f.bin").read_bytes())
    # corrupt native 1; list all chunks: decoder must skip it and still rebuild the file
    bad = bytearray((tmp_path / "_1_f.bin").read_bytes())
    bad[100] ^= 0xFF
    (tmp_path / "_1_f.bin").write_bytes(bytes(bad))
    ff.write_conf(str(tmp_path / "conf"), [ff.chunk_path(str(f), i) for i in range(7)])
    r = cpu().decode_file(str(f), str(tmp_path / "conf"), str(tmp_path / "o"))
    assert r["rejected"] == 1 and (tmp_path / "o").read_bytes() == payload


def test_aggressive_read_skips_missing_and_singular_subsets(tmp_path):
    f = tmp_path / "f.bin"
    payload = os.urandom(33_333)
    f.write_bytes(payload)
    cpu().encode_file(str(f), 10, 4)
    g = GF256.generator(GF256.vandermonde_ref(10, 4))
    bad = list(GF256.singular_patterns(g, 10)[0])  # a singular first-k subset ...
    rest = [r for r in range(14) if r not in bad]
    os.remove(tmp_path / f"_{rest[0]}_f.bin")  # ... plus one missing chunk listed after it
    ff.write_conf(str(tmp_path / "conf"), [ff.chunk_path(str(f), r) for r in bad + rest])
    cpu().decode_file(str(f), str(tmp_path / "conf"), str(tmp_path / "o"))
    assert (tmp_path / "o").read_bytes() == payload


def test_plan_cache_is_lru():
    from gpu_rscode_amd.models.rs import _PlanCache

    c = _PlanCache(capacity=3)
    for i in range(3):
        c[i] = i
    assert c.get(0) == 0  # 0 becomes the most recent
    c[3] = 3  # evicts 1, the least recently used
    assert list(c) == [2, 0, 3] and c.get(1) is None


def test_row_pitch_layout(monkeypatch):
    """alloc_rows / row_pitch: every pitch a multiple of 256 (16-byte aligned rows for odd C);
    device rows of >= 8 MiB rounded to 2 MiB (measured HBM placement win), host rows never; pitches
    that are multiples of 64 MiB skewed by a quarter; GFRS_TUNE=row_align / row_skew override."""
    from gpu_rscode_amd.models.rs import alloc_rows, row_pitch
    C = 107374183  # the headline chunk (1 GiB / 10, odd)
    assert row_pitch(C, "cpu") == 107374336
    assert row_pitch(C, "cuda") % (2 << 20) == 0 and row_pitch(C, "cuda") >= C
    assert row_pitch(1000, "cuda") == 1024 and row_pitch(1, "cuda") == 256
    assert row_pitch((8 << 20) - 1, "cuda") == 8 << 20
    # a pitch that is a multiple of 64 MiB gets a quarter more (HBM channel placement of large rows)
    assert row_pitch(512 << 20, "cuda") == 640 << 20 and row_pitch(128 << 20, "cuda") == 160 << 20
    assert row_pitch((512 << 20) - 5, "cuda") == 640 << 20 and row_pitch(C, "cuda") == 104 << 20
    assert row_pitch(512 << 20, "cpu") == 512 << 20
    monkeypatch.setenv("GFRS_TUNE", "row_skew=8388608")
    assert row_pitch(512 << 20, "cuda") == 520 << 20
    monkeypatch.setenv("GFRS_TUNE", "row_skew=0")
    assert row_pitch(512 << 20, "cuda") == 512 << 20
    monkeypatch.setenv("GFRS_TUNE", "row_align=256")
    assert row_pitch(C, "cuda") == 107374336
    t = alloc_rows(3, 1001, "cpu", fill=7)
    assert t.shape == (3, 1001) and t.stride() == (1024, 1) and int(t.sum()) == 7 * 3 * 1001


def test_flat_rows_view_starts_at_the_rows():
    """flat_rows covers exactly the rows (pitch included) from the tensor's own storage offset."""
    from gpu_rscode_amd import flat_rows
    base = torch.arange(5000, dtype=torch.int64).to(torch.uint8)
    t = base.as_strided((3, 1000), (1024, 1), 700)
    f = flat_rows(t)
    assert f.shape == (3072,) and f.data_ptr() == t.data_ptr()
    assert torch.equal(f[1024:2024], t[1])
