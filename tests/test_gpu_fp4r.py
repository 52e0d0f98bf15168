"""GF(2^8) on the FP4 matrix cores, register-streamed form (csrc/kernels/gf_mfma8r.hip), against the
numpy GF(2^8) oracle: uniform-stride and scattered inputs, fused survivor copies, ragged and odd
tails, column sub-ranges, every M-tile grouping, and a device-built decode plan."""
import numpy as np
import pytest
import torch

from gpu_rscode_amd import gf
from gpu_rscode_amd.models import ReedSolomon, alloc_rows
from gpu_rscode_amd.ops import GemmPlan

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _form_r(monkeypatch):
    monkeypatch.setenv("GFRS_FP4_FORM", "r")


def _rand(rows, C, seed):
    return torch.from_numpy(np.random.default_rng(seed).integers(0, 256, size=(rows, C), dtype=np.uint8))


@pytest.mark.parametrize("k,m,C,scattered,col", [
    (128, 32, 512 * 64, False, (0, None)),
    (128, 26, 512 * 37 + 301, True, (0, None)),   # 7 M-tiles, odd tail
    (64, 12, 512 * 9 + 2, False, (2, 512 * 8 + 7)),  # 3 M-tiles, sub-range with an odd end
    (20, 4, 1000, True, (0, None)),                # one tile, one partial chunk
    (255, 8, 512 * 4, False, (512, 1024)),         # k past 2 x 128 (still one pass)
])
def test_fp4r_matches_oracle(k, m, C, scattered, col):
    rng = np.random.default_rng(k * 7 + m)
    coeff = rng.integers(0, 256, size=(m, k), dtype=np.uint8)
    coeff[0, :3] = [0, 1, 255]
    x = alloc_rows(k, C, "cuda")
    x.copy_(_rand(k, C, C))
    inputs = [x[i].clone() for i in range(k)] if scattered else x
    y = alloc_rows(m, C, "cuda", fill=0x5A)
    plan = GemmPlan(inputs, y, coeff, engine="mfma")
    assert plan.engine == "mfma" and plan.fp4_form == "r"
    c0, n = col[0], (C - col[0] if col[1] is None else col[1])
    plan.run(col0=c0, ncols=n)
    torch.cuda.synchronize()
    want = gf.GF256.gemm(coeff, x.cpu().numpy())
    got = y.cpu().numpy()
    assert np.array_equal(got[:, c0:c0 + n], want[:, c0:c0 + n])
    assert (got[:, :c0] == 0x5A).all() and (got[:, c0 + n:] == 0x5A).all()


@pytest.mark.parametrize("mg", ["1", "2", "3", "4"])
def test_fp4r_every_grouping_with_copies(mg, monkeypatch):
    """Decode shape (26 rebuilt, 102 copied) at each forced M-tile grouping: outputs and copies."""
    monkeypatch.setenv("GFRS_FP4R_MG", mg)  # read when the plan is built
    k, m, C = 128, 26, 512 * 21 + 77
    rng = np.random.default_rng(11)
    coeff = rng.integers(0, 256, size=(m, k), dtype=np.uint8)
    x = alloc_rows(k, C, "cuda")
    x.copy_(_rand(k, C, 3))
    inputs = [x[i] for i in range(k)]
    y = alloc_rows(m, C, "cuda", fill=0)
    dst = alloc_rows(k, C, "cuda", fill=0)
    copies = [dst[i] if i % 5 else None for i in range(k)]
    plan = GemmPlan(inputs, y, coeff, copies=copies, engine="mfma")
    plan.run()
    torch.cuda.synchronize()
    assert np.array_equal(y.cpu().numpy(), gf.GF256.gemm(coeff, x.cpu().numpy()))
    xd, dd = x.cpu().numpy(), dst.cpu().numpy()
    for i in range(k):
        assert np.array_equal(dd[i], xd[i] if i % 5 else np.zeros(C, np.uint8))


def test_fp4r_device_built_decode():
    """ReedSolomon.decode(device_invert=True) on the r form: the bit-matrix comes from the
    device-solved decode rows (set_device_coeff), survivors copied in the same pass."""
    k, n, C = 128, 160, 512 * 40 + 33
    rs = ReedSolomon(k, n, matrix="cauchy")
    data = alloc_rows(k, C, "cuda")
    data.copy_(_rand(k, C, 9))
    par = rs.encode(data)
    rng = np.random.default_rng(2)
    erased = set(rng.choice(n, size=n - k, replace=False).tolist())
    rows = [r for r in range(n) if r not in erased]
    stripe = [data[r] if r < k else par[r - k] for r in rows]
    out = alloc_rows(k, C, "cuda", fill=0)
    rs.decode(stripe, rows, out=out, device_invert=True)
    torch.cuda.synchronize()
    assert torch.equal(out, data)
