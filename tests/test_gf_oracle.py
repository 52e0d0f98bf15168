"""GF(2^w) oracle and coding-matrix tests (CPU).

Golden vectors: the slide deck's worked inverse (doc/slide.tex:551-556), the blocked
Gauss-Jordan test matrix of src/decode-gj.cu:1282 with its expected inverse at :1453, and the
k=10,p=4 reference Vandermonde (verified against src/cpu-rs.c:446-457).
"""
import itertools

import numpy as np
import pytest

from gpu_rscode_amd import gf
from gpu_rscode_amd.gf import GF, GF256, SingularMatrixError


def test_field_tables_reference_layout():
    # exp/log in the reference's zero-band layout: exp[0..510) two periods, log(0)=510
    exp = GF256.exp
    assert exp[0] == 1 and exp[1] == 2 and exp[8] == 0x1D  # x^8 = x^4+x^3+x^2+1
    assert all(exp[i] == exp[i + 255] for i in range(255))
    assert sorted(exp[:255].tolist()) == list(range(1, 256))


def test_native_tables_match_oracle():
    from gpu_rscode_amd._native import cpu

    t = cpu().tables()
    ex = np.frombuffer(t["exp"], dtype=np.uint8)
    assert len(ex) == 1021
    assert np.array_equal(ex[:510], GF256.exp[:510].astype(np.uint8))
    assert not ex[510:].any()
    lg = np.array(t["log"])
    assert lg[0] == 510
    assert np.array_equal(lg[1:], GF256.log[1:])


def test_mul_div_inverse_properties():
    a = np.arange(256)
    for c in (1, 2, 3, 0x53, 0xCA, 255):
        prod = GF256.mul(a, c)
        assert sorted(prod[1:].tolist()) == list(range(1, 256))  # multiplication by c != 0 is a bijection
        assert np.array_equal(GF256.div(prod, c), a)
    # agree with the bitwise shift-and-xor definition over poly 0x11D
    def slow(x, y):
        r = 0
        for i in range(8):
            if y >> i & 1:
                r ^= x
            x <<= 1
            if x & 0x100:
                x ^= 0x11D
        return r
    for x, y in itertools.product(range(0, 256, 7), range(0, 256, 11)):
        assert GF256.mul(x, y) == slow(x, y)


def test_pow_ref_quirk():
    assert GF256.pow_ref(0, 3) == 1  # reference gf_pow(0, e) == 1 (src/matrix.cu:204-208)
    assert GF256.pow(0, 3) == 0
    assert GF256.pow_ref(2, 8) == 0x1D


def test_vandermonde_ref_k10_p4_golden():
    e = GF256.vandermonde_ref(10, 4)
    assert e[0].tolist() == [1] * 10
    assert e[1].tolist() == list(range(1, 11))
    assert e[2].tolist() == [1, 4, 5, 16, 17, 20, 21, 64, 65, 68]
    assert e[3].tolist() == [1, 8, 15, 64, 85, 120, 107, 58, 115, 146]


def test_inverse_golden_slides_and_decode_gj():
    a = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [1, 2, 3, 4], [1, 1, 1, 1]])
    inv = GF256.invert(a)
    assert inv[2].tolist() == [104, 187, 186, 210] and inv[3].tolist() == [105, 186, 186, 211]
    b = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [1, 1, 1, 1], [1, 2, 3, 4]])
    inv = GF256.invert(b)
    assert inv[2].tolist() == [104, 187, 210, 186] and inv[3].tolist() == [105, 186, 211, 186]
    assert np.array_equal(GF256.matmul(b, inv), np.eye(4, dtype=np.uint8))


def test_singular_census_matches_survey():
    # the reference [I;V] generator is not MDS
    for (k, p), expect in {(4, 2): 0, (4, 3): 0, (10, 4): 12}.items():
        g = GF256.generator(GF256.vandermonde_ref(k, p))
        bad = GF256.singular_patterns(g, k)
        assert len(bad) == expect, (k, p, len(bad))
    g = GF256.generator(GF256.vandermonde_ref(10, 4))
    erasure_sets = sorted(tuple(sorted(set(range(14)) - set(s))) for s in GF256.singular_patterns(g, 10))
    assert (4, 5, 9, 11) in erasure_sets and (0, 1, 2, 12) in erasure_sets


@pytest.mark.parametrize("kind", ["cauchy", "sys_vandermonde"])
def test_mds_constructions(kind):
    k, p = 6, 3
    g = GF256.generator(GF256.encoding_matrix(kind, k, p))
    assert GF256.singular_patterns(g, k) == []


def test_invert_singular_raises():
    with pytest.raises(SingularMatrixError):
        GF256.invert(np.array([[1, 2], [2, 4]]))


def test_gf16_tables_match_reference_header():
    # src/gf16.h: poly x^4+x+1 exp table
    f = GF(4)
    assert f.exp[:15].tolist() == [1, 2, 4, 8, 3, 6, 12, 11, 5, 10, 7, 14, 15, 13, 9]
    assert f.mul(7, 9) == f.exp[(f.log[7] + f.log[9]) % 15]


def test_gf65536_field():
    f = GF(16)
    x = np.array([1, 2, 0x1234, 0xFFFF])
    assert np.array_equal(f.div(f.mul(x, 0xBEEF), 0xBEEF), x)


def test_perm_records_reproduce_every_product():
    x = np.arange(256, dtype=np.uint8)
    for c in range(256):
        rec = gf.perm_record(gf.byte_map_gf256(c))
        assert np.array_equal(gf.perm_apply(rec, x), gf.byte_map_gf256(c)), c


def test_perm_records_native_equal_python():
    from gpu_rscode_amd._native import cpu

    for c in (0, 1, 2, 29, 142, 255):
        assert list(cpu().perm_table(c)) == gf.perm_record(gf.byte_map_gf256(c)).tolist()


def test_gf16_nibble_maps_are_linear():
    for c in range(16):
        assert gf.is_linear(gf.byte_map_gf16_nibbles(c))
        rec = gf.perm_record(gf.byte_map_gf16_nibbles(c))
        assert np.array_equal(gf.perm_apply(rec, np.arange(256)), gf.byte_map_gf16_nibbles(c))


def test_auto_engine_policy():
    from gpu_rscode_amd.ops.gemm import _auto_engine
    assert _auto_engine(128, 32, True, False, 1) == "mfma"
    assert _auto_engine(64, 16, True, False, 1) == "mfma"
    assert _auto_engine(10, 4, True, False, 1) == "valu"  # narrow: v_perm is at the HBM roofline
    assert _auto_engine(128, 32, False, False, 1) == "valu"  # GF(16) nibble maps
    assert _auto_engine(128, 32, True, True, 1) == "valu"  # unaligned rows
    assert _auto_engine(128, 32, True, False, 4) == "valu"  # batched stripes


def test_trace_ranges_are_safe_without_profiler():
    from gpu_rscode_amd._native import cpu
    from gpu_rscode_amd.utils.timing import trace_range
    assert isinstance(cpu().roctx_available(), bool)
    with trace_range("test/outer"):
        with trace_range("test/inner"):
            cpu().trace_mark("test/mark")
