"""Property-based tests (hypothesis): GF(2^8) field laws, codec round trips and linearity over
random (k, n, C, erasure pattern), on the C++ CPU codec and on the HIP kernels.

The reference has no test suite; its decode contract — any k surviving chunks of an
MDS code give back the file (`src/decode.cu:302-333`) — is checked here for random shapes instead
of the fixed ones in test_cpu_codec.py / test_gpu_codec.py. Every oracle is the numpy GF(2^8)
model in gpu_rscode_amd/gf.py. Runs are derandomized, so a failure reproduces exactly.
"""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, example, given, settings
from hypothesis import strategies as st

from gpu_rscode_amd import ReedSolomon, UnrecoverableError, alloc_rows
from gpu_rscode_amd.gf import GF256
from gpu_rscode_amd._native import cpu

CPU_SETTINGS = settings(max_examples=60, deadline=None, derandomize=True,
                        suppress_health_check=[HealthCheck.too_slow])
GPU_SETTINGS = settings(max_examples=20, deadline=None, derandomize=True,
                        suppress_health_check=[HealthCheck.too_slow])
byte = st.integers(0, 255)
nonzero = st.integers(1, 255)


@st.composite
def code_case(draw, k_max=24, p_max=8, c_max=777, mds=True):
    """(k, p, C, matrix, survivor rows, seed) with a random k-subset of the n chunks."""
    k = draw(st.integers(1, k_max))
    p = draw(st.integers(0, p_max))
    C = draw(st.integers(1, c_max))
    matrix = draw(st.sampled_from(["cauchy", "sys_vandermonde"] if mds else ["vandermonde"]))
    rows = sorted(draw(st.permutations(range(k + p)))[:k])
    return k, p, C, matrix, rows, draw(st.integers(0, 2**31))


# ---- field laws (numpy oracle and the native constexpr tables) ---------------------------------
@CPU_SETTINGS
@given(byte, byte, byte)
def test_field_laws(a, b, c):
    mul = GF256.mul
    assert mul(a, b) == mul(b, a)
    assert mul(mul(a, b), c) == mul(a, mul(b, c))
    assert mul(a, b ^ c) == mul(a, b) ^ mul(a, c)
    assert mul(a, 1) == a and mul(a, 0) == 0


@CPU_SETTINGS
@given(byte, nonzero)
def test_native_mul_div_match_oracle(a, b):
    assert cpu().mul(a, b) == GF256.mul(a, b)
    assert cpu().div(a, b) == GF256.div(a, b)
    assert GF256.mul(cpu().div(a, b), b) == a
    assert GF256.mul(b, GF256.inv(b)) == 1


@CPU_SETTINGS
@given(st.integers(1, 12), st.integers(0, 2**31))
def test_invert_is_inverse(n, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 256, size=(n, n), dtype=np.uint8)
    if not GF256.is_invertible(a):
        return
    inv = GF256.invert(a)
    assert np.array_equal(GF256.matmul(a, inv), np.eye(n, dtype=np.uint8))


# ---- CPU codec ---------------------------------------------------------------------------------
def _cpu_rows(k, C, seed):
    host = np.random.default_rng(seed).integers(0, 256, size=(k, C), dtype=np.uint8)
    return host, torch.from_numpy(host.copy())


@CPU_SETTINGS
@given(code_case())
def test_cpu_encode_decode_roundtrip_mds(case):
    k, p, C, matrix, rows, seed = case
    rs = ReedSolomon(k, k + p, matrix=matrix)
    host, data = _cpu_rows(k, C, seed)
    parity = rs.encode(data)
    assert np.array_equal(parity.numpy(), GF256.gemm(rs.E, host))
    stripe = [data[i] for i in range(k)] + [parity[i] for i in range(p)]
    out = rs.decode(torch.stack([stripe[r] for r in rows]), rows)
    assert np.array_equal(out.numpy(), host)


@CPU_SETTINGS
@given(code_case(mds=False))
def test_cpu_reference_vandermonde_decodes_or_flags(case):
    """The reference [I; V] is not MDS: every pattern either decodes exactly or is
    reported unrecoverable — never silently wrong."""
    k, p, C, matrix, rows, seed = case
    rs = ReedSolomon(k, k + p, matrix=matrix)
    host, data = _cpu_rows(k, C, seed)
    parity = rs.encode(data)
    stripe = [data[i] for i in range(k)] + [parity[i] for i in range(p)]
    survivors = torch.stack([stripe[r] for r in rows])
    if rs.is_recoverable(rows):
        assert np.array_equal(rs.decode(survivors, rows).numpy(), host)
    else:
        with pytest.raises(UnrecoverableError):
            rs.decode(survivors, rows)


@CPU_SETTINGS
@given(code_case(p_max=6), st.data())
def test_cpu_reconstruct_rewrites_erased_rows(case, draw):
    k, p, C, matrix, _, seed = case
    rs = ReedSolomon(k, k + p, matrix=matrix)
    host, data = _cpu_rows(k, C, seed)
    stripe = torch.cat([data, rs.encode(data)])
    want = stripe.clone()
    erased = draw.draw(st.lists(st.integers(0, k + p - 1), max_size=p, unique=True))
    stripe[erased] = 0
    rs.reconstruct(stripe, erased)
    assert torch.equal(stripe, want)


@CPU_SETTINGS
@given(st.integers(1, 16), st.integers(1, 6), st.integers(1, 300), st.integers(0, 2**31))
def test_cpu_encode_is_linear(k, p, C, seed):
    rs = ReedSolomon(k, k + p)
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 256, size=(k, C), dtype=np.uint8)
    b = rng.integers(0, 256, size=(k, C), dtype=np.uint8)
    pa, pb, pab = (rs.encode(torch.from_numpy(x)).numpy() for x in (a, b, a ^ b))
    assert np.array_equal(pa ^ pb, pab)
    assert rs.verify(torch.from_numpy(a), torch.from_numpy(pa))


# ---- HIP kernels -------------------------------------------------------------------------------
@pytest.mark.gpu
@GPU_SETTINGS
@given(code_case(k_max=140, p_max=40, c_max=70_000), st.booleans())
@example(case=(100, 20, 12345, "cauchy", list(range(20, 120)), 7), device_invert=True)  # FP4 both ways
def test_gpu_encode_decode_roundtrip(case, device_invert):
    """Random shapes through the auto engine: v_perm for narrow codes, FP4 MFMA for k >= 64, m >= 16."""
    k, p, C, matrix, rows, seed = case
    rs = ReedSolomon(k, k + p, matrix=matrix)
    host = np.random.default_rng(seed).integers(0, 256, size=(k, C), dtype=np.uint8)
    data = alloc_rows(k, C, "cuda")
    data.copy_(torch.from_numpy(host))
    parity = rs.encode(data)
    stripe = [data[i] for i in range(k)] + [parity[i] for i in range(p)]
    out = rs.decode([stripe[r] for r in rows], rows, device_invert=device_invert)
    torch.cuda.synchronize()
    if device_invert and any(r >= k for r in rows):
        assert int(rs.last_status.item()) == 0
    assert np.array_equal(parity.cpu().numpy(), GF256.gemm(rs.E, host)), (k, p, C)
    assert np.array_equal(out.cpu().numpy(), host), (k, p, C, rows)


@pytest.mark.gpu
@GPU_SETTINGS
@given(st.integers(1, 4), code_case(k_max=16, p_max=6, c_max=5000))
def test_gpu_encode_batch_matches_oracle(batch, case):
    k, p, C, matrix, _, seed = case
    if p == 0:
        return
    rs = ReedSolomon(k, k + p, matrix=matrix)
    host = np.random.default_rng(seed).integers(0, 256, size=(batch, k, C), dtype=np.uint8)
    parity = rs.encode_batch(torch.from_numpy(host).cuda())
    torch.cuda.synchronize()
    for b in range(batch):
        assert np.array_equal(parity[b].cpu().numpy(), GF256.gemm(rs.E, host[b]))


# ---- GF(2^16) (the reference's w = 16 field) -----------------------------------------------------
F16 = None


def _f16():
    global F16
    if F16 is None:
        from gpu_rscode_amd.gf import field
        F16 = field(16)
    return F16


@CPU_SETTINGS
@given(st.integers(0, 65535), st.integers(0, 65535), st.integers(1, 65535))
def test_gf65536_native_mul_and_byte_maps(a, b, c):
    from gpu_rscode_amd.gf import perm_quads16, quad_apply16

    f = _f16()
    assert cpu().gf16_mul(a, b) == int(f.mul(a, b))
    q = perm_quads16(np.array([[c]]))[0, 0]
    x = np.array([a, b], dtype=np.uint16)
    assert np.array_equal(quad_apply16(q, x), f.mul(c, x).astype(np.uint16))


@st.composite
def code16_case(draw, k_max=40, p_max=12, s_max=300):
    k = draw(st.integers(1, k_max))
    p = draw(st.integers(0, p_max))
    C = 2 * draw(st.integers(1, s_max))  # whole 16-bit symbols
    matrix = draw(st.sampled_from(["cauchy", "sys_vandermonde"]))
    rows = sorted(draw(st.permutations(range(k + p)))[:k])
    return k, p, C, matrix, rows, draw(st.integers(0, 2**31))


@settings(max_examples=25, deadline=None, derandomize=True, suppress_health_check=[HealthCheck.too_slow])
@given(code16_case())
def test_cpu_gf65536_roundtrip_mds(case):
    k, p, C, matrix, rows, seed = case
    rs = ReedSolomon(k, k + p, matrix=matrix, field="gf65536")
    host, data = _cpu_rows(k, C, seed)
    parity = rs.encode(data)
    assert np.array_equal(parity.numpy().view("<u2"), _f16().gemm(rs.E, host.view("<u2")))
    stripe = [data[i] for i in range(k)] + [parity[i] for i in range(p)]
    out = rs.decode(torch.stack([stripe[r] for r in rows]), rows)
    assert np.array_equal(out.numpy(), host)


@pytest.mark.gpu
@GPU_SETTINGS
@given(code16_case(k_max=300, p_max=40, s_max=20_000), st.booleans())
@example(case=(300, 40, 2 * 4099, "cauchy", list(range(40, 340)), 11), aligned=False)
def test_gpu_gf65536_roundtrip(case, aligned):
    """Random GF(2^16) shapes on the device kernel (vector kernel on pitched rows, the symbol kernel
    on rows 2 bytes off a 16-byte boundary), bit-exact against the numpy oracle."""
    k, p, C, matrix, rows, seed = case
    rs = ReedSolomon(k, k + p, matrix=matrix, field="gf65536")
    host = np.random.default_rng(seed).integers(0, 256, size=(k, C), dtype=np.uint8)
    if aligned:
        data = alloc_rows(k, C, "cuda")
        data.copy_(torch.from_numpy(host))
        drows = [data[i] for i in range(k)]
    else:
        flat = torch.zeros(k * (C + 2) + 2, dtype=torch.uint8, device="cuda")
        drows = [flat[2 + i * (C + 2): 2 + i * (C + 2) + C] for i in range(k)]
        for i in range(k):
            drows[i].copy_(torch.from_numpy(host[i]))
    parity = alloc_rows(p, C, "cuda") if p else None
    if p:
        rs.encode(drows, parity)
    stripe = drows + ([parity[i] for i in range(p)] if p else [])
    out = rs.decode([stripe[r] for r in rows], rows)
    torch.cuda.synchronize()
    if p:
        assert np.array_equal(parity.cpu().numpy().view("<u2"), _f16().gemm(rs.E, host.view("<u2"))), (k, p, C)
    assert np.array_equal(out.cpu().numpy(), host), (k, p, C, rows)
