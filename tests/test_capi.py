"""The C API (csrc/include/gfrs.h, lib/libgfrs.so): the header is plain C99 and C++, the library
exports exactly the header's functions and nothing else, the host matrix functions agree with the
numpy GF(2^8) oracle through ctypes, and (GPU) the C demo and the file codec run end to end."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from gpu_rscode_amd import _build, gf
from gpu_rscode_amd.models import ReedSolomon

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "csrc", "include", "gfrs.h")
LIB = os.path.join(ROOT, "lib", "libgfrs.so")
DEMO = os.path.join(ROOT, "bin", "gfrs_capi_demo")


@pytest.fixture(scope="module")
def lib():
    if _build.have_sources() and (_build.stale(_build.Path(LIB)) or not os.path.exists(DEMO)):
        _build.build("capi")
    return ctypes.CDLL(LIB)


def _declared() -> set[str]:
    text = open(HEADER).read()
    return set(re.findall(r"\b(gfrs_[a-z_0-9]+)\s*\(", text))


@pytest.mark.parametrize("compiler,flags", [("gcc", ["-x", "c", "-std=c99", "-pedantic"]),
                                            ("g++", ["-x", "c++", "-std=c++17"])])
def test_header_compiles_standalone(compiler, flags, tmp_path):
    src = tmp_path / "use.c"
    src.write_text('#include "gfrs.h"\nint main(void) { return gfrs_api_version() == GFRS_API_VERSION ? 0 : 1; }\n')
    r = subprocess.run([compiler, *flags, "-Wall", "-Werror", "-fsyntax-only", f"-I{os.path.dirname(HEADER)}",
                        str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_library_exports_exactly_the_header(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    assert exported == _declared()


def test_encoding_and_decode_matrices_match_the_oracle(lib):
    k, p = 10, 4
    e = np.zeros((p, k), dtype=np.uint8)
    buf = e.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
    assert lib.gfrs_encoding_matrix(0, k, p, buf) == 0
    assert np.array_equal(e, ReedSolomon(k, k + p).E)  # the reference's Vandermonde
    for kind, name in ((1, "cauchy"), (2, "sys_vandermonde")):
        m = np.zeros((p, k), dtype=np.uint8)
        assert lib.gfrs_encoding_matrix(kind, k, p, m.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))) == 0
        assert np.array_equal(m, gf.GF256.encoding_matrix(name, k, p)), name
    rows = np.array([0, 2, 3, 5, 6, 8, 9, 10, 12, 13], dtype=np.int32)
    dm = np.zeros((k, k), dtype=np.uint8)
    rc = lib.gfrs_decode_matrix(buf, k, p, rows.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                dm.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    assert rc == 0
    g = np.vstack([np.eye(k, dtype=np.uint8), e])
    assert np.array_equal(gf.GF256.gemm(dm, g[rows]), np.eye(k, dtype=np.uint8))
    # a repeated survivor is singular; an out-of-range id is an argument error with a message
    bad = rows.copy()
    bad[1] = bad[0]
    assert lib.gfrs_decode_matrix(buf, k, p, bad.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                  dm.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))) == -2
    bad[1] = 99
    assert lib.gfrs_decode_matrix(buf, k, p, bad.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                  dm.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))) == -1
    lib.gfrs_last_error.restype = ctypes.c_char_p
    assert b"out of range" in lib.gfrs_last_error()


def test_bad_arguments_are_reported_not_crashed(lib):
    lib.gfrs_last_error.restype = ctypes.c_char_p
    assert lib.gfrs_encoding_matrix(0, 200, 100, None) == -1
    assert lib.gfrs_encode_file(None, 10, 4, 0, None, 0, 2, None) == -1
    assert b"no file" in lib.gfrs_last_error()
    plan = ctypes.c_void_p()
    assert lib.gfrs_plan_create(ctypes.byref(plan), 0, 0, 4, None, None, None, None, 0, 0) == -1


@pytest.mark.gpu
def test_gpu_capi_demo(lib):
    """csrc/capi/demo.c: encode plan, device-built decoder (valid, invalid, singular patterns),
    a k=128 p=32 stripe on the FP4 matrix-core engine and the host pipeline, all from C."""
    r = subprocess.run([DEMO], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "capi_demo OK" in r.stdout and "engine=mfma" in r.stdout


@pytest.mark.gpu
def test_gpu_capi_file_codec_round_trip(lib, tmp_path):
    """gfrs_encode_file / gfrs_decode_file (the reference's two C entry points) on a 3 MB file with
    the first four natives erased (src/unit-test.sh's pattern)."""
    data = np.random.default_rng(3).integers(0, 256, size=3_000_017, dtype=np.uint8).tobytes()
    f = tmp_path / "obj.bin"
    f.write_bytes(data)

    class Report(ctypes.Structure):
        _fields_ = [("total_size", ctypes.c_int64), ("chunk_size", ctypes.c_int64), ("k", ctypes.c_int),
                    ("p", ctypes.c_int), ("erased", ctypes.c_int), ("rejected", ctypes.c_int),
                    ("ms_alloc", ctypes.c_double), ("ms_read", ctypes.c_double), ("ms_matrix", ctypes.c_double),
                    ("ms_compute", ctypes.c_double), ("ms_write", ctypes.c_double)]

    rep = Report()
    lib.gfrs_last_error.restype = ctypes.c_char_p
    assert lib.gfrs_encode_file(str(f).encode(), 10, 4, 0, None, 0, 2, ctypes.byref(rep)) == 0, lib.gfrs_last_error()
    assert rep.k == 10 and rep.p == 4 and rep.total_size == len(data)
    conf = tmp_path / "conf"
    conf.write_text("".join(f"{tmp_path}/_{i}_obj.bin\n" for i in range(4, 14)))
    out = tmp_path / "out.bin"
    assert lib.gfrs_decode_file(str(f).encode(), str(conf).encode(), str(out).encode(), None, 0, 2,
                                ctypes.byref(rep)) == 0, lib.gfrs_last_error()
    assert rep.erased == 4 and out.read_bytes() == data
    assert lib.gfrs_release() == 0


@pytest.mark.gpu
def test_gpu_capi_file_codec_ex_gf65536_zero_copy(lib, tmp_path):
    """gfrs_encode_file_ex / gfrs_decode_file_ex (API version 2): a GF(2^16) stripe of 300 + 40
    chunks (past GF(2^8)'s 256) encoded and decoded with the zero-copy kernel path."""
    data = np.random.default_rng(5).integers(0, 256, size=2_000_011, dtype=np.uint8).tobytes()
    f = tmp_path / "obj.bin"
    f.write_bytes(data)
    lib.gfrs_last_error.restype = ctypes.c_char_p
    assert lib.gfrs_api_version() >= 2
    assert lib.gfrs_encode_file_ex(str(f).encode(), 300, 40, 1, 16, 1, None, 0, 2, None) == 0, lib.gfrs_last_error()
    assert open(str(f) + ".METADATA").readline() == "GFRS-METADATA 2 16\n"
    conf = tmp_path / "conf"
    conf.write_text("".join(f"{tmp_path}/_{i}_obj.bin\n" for i in range(40, 340)))
    out = tmp_path / "out.bin"
    assert lib.gfrs_decode_file_ex(str(f).encode(), str(conf).encode(), str(out).encode(), 1, None, 0, 2,
                                   None) == 0, lib.gfrs_last_error()
    assert out.read_bytes() == data
    assert lib.gfrs_encode_file_ex(str(f).encode(), 4, 2, 0, 12, 0, None, 0, 2, None) == -1  # bad field width
    assert lib.gfrs_release() == 0


def test_gf65536_matrices_match_the_oracle(lib):
    """API version 3: gfrs_encoding_matrix16 equals ReedSolomon(field="gf65536")'s E for every kind,
    and gfrs_decode_rows16 rebuilds the erased natives (oracle: rows of G applied to the data)."""
    F = gf.field(16)
    k, p = 12, 5
    for kind, name in ((0, "vandermonde"), (1, "cauchy"), (2, "sys_vandermonde")):
        e = np.zeros((p, k), dtype=np.uint16)
        assert lib.gfrs_encoding_matrix16(kind, k, p, e.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16))) == 0
        assert np.array_equal(e.astype(np.int64), np.asarray(ReedSolomon(k, k + p, field="gf65536", matrix=name).E))
    e = np.zeros((p, k), dtype=np.uint16)
    assert lib.gfrs_encoding_matrix16(1, k, p, e.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16))) == 0
    data = np.random.default_rng(2).integers(0, 65536, size=(k, 33)).astype(np.int64)
    chunks = np.concatenate([data, F.gemm(e.astype(np.int64), data)])
    erased = [1, 4, 9]
    rows = [r for r in range(k + p) if r not in erased][:k]
    out = np.zeros((len(erased), k), dtype=np.uint16)
    rc = lib.gfrs_decode_rows16(e.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)), k, p,
                                np.asarray(rows, dtype=np.int32).ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                np.asarray(erased, dtype=np.int32).ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                len(erased), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)))
    assert rc == 0
    assert np.array_equal(F.gemm(out.astype(np.int64), chunks[rows]), data[erased])
    bad = np.asarray([0] * k, dtype=np.int32)  # repeated survivor: not recoverable
    assert lib.gfrs_decode_rows16(e.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)), k, p,
                                  bad.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                  np.asarray(erased, dtype=np.int32).ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                  len(erased), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16))) in (-1, -2)


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,C,engine", [(300, 40, 2 * 4096 + 100, 0), (10, 4, 2 * 5000, 0), (64, 16, 8192, 1),
                                          (64, 16, 8192, 2)])
def test_gpu_capi_plan16_matches_oracle(lib, k, m, C, engine):
    """gfrs_plan16_*: the GF(2^16) device GEMM through the C API, on the matrix cores (AUTO for
    k >= 16, or MFMA) and the v_perm kernel (AUTO at k = 10, or VALU), against the numpy oracle."""
    import torch

    from gpu_rscode_amd.models import alloc_rows

    F = gf.field(16)
    rng = np.random.default_rng(k + m)
    coeff = rng.integers(0, 65536, size=(m, k)).astype(np.uint16)
    x = alloc_rows(k, C, "cuda")
    x.copy_(torch.from_numpy(rng.integers(0, 256, size=(k, C), dtype=np.uint8)))
    y = alloc_rows(m, C, "cuda", fill=0)
    ins = (ctypes.c_void_p * k)(*[int(x[i].data_ptr()) for i in range(k)])
    outs = (ctypes.c_void_p * m)(*[int(y[i].data_ptr()) for i in range(m)])
    plan = ctypes.c_void_p()
    lib.gfrs_last_error.restype = ctypes.c_char_p
    torch.cuda.synchronize()
    rc = lib.gfrs_plan16_create(ctypes.byref(plan), 0, k, m, coeff.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)),
                                ins, outs, None, ctypes.c_int64(C), engine)
    assert rc == 0, lib.gfrs_last_error()
    want_engine = engine or (2 if k >= 16 else 1)
    assert lib.gfrs_plan16_engine(plan) == want_engine
    assert lib.gfrs_plan16_run(plan, None) == 0
    assert lib.gfrs_sync(0) == 0
    got = y.cpu().numpy().view("<u2").astype(np.int64)
    assert np.array_equal(got, F.gemm(coeff.astype(np.int64), np.ascontiguousarray(x.cpu().numpy()).view("<u2")))
    lib.gfrs_plan16_destroy(plan)
