"""gfx950 kernel numerics vs the numpy GF oracle (GPU)."""
import numpy as np
import pytest
import torch

from gpu_rscode_amd import gf
from gpu_rscode_amd.gf import GF256
from gpu_rscode_amd.models import alloc_rows
from gpu_rscode_amd.ops import GemmPlan, fill_random_, gen_matrix_device, gf_invert, invert_into_plan
from gpu_rscode_amd.ops.gemm import perm_tables_from_coeff
from gpu_rscode_amd.utils.tune import with_tune

pytestmark = pytest.mark.gpu


def _native_loaded():
    from gpu_rscode_amd._native import hip

    h = hip()
    assert h.device_count() > 0, "HIP module loaded but sees no device"
    return h


def _rand_rows(rows, ncols, seed, device="cuda"):
    g = np.random.default_rng(seed)
    host = g.integers(0, 256, size=(rows, ncols), dtype=np.uint8)
    t = alloc_rows(rows, ncols, device)
    t.copy_(torch.from_numpy(host))
    return host, t


@pytest.mark.parametrize("k,m,ncols", [(4, 2, 1 << 16), (10, 4, 1000003), (10, 4, 4096 + 7), (16, 4, 65536),
                                        (3, 1, 17), (1, 1, 1), (8, 8, 12345), (12, 16, 40000), (32, 20, 7777),
                                        (128, 32, 20000), (5, 3, 15)])
def test_gemm_matches_oracle(k, m, ncols):
    _native_loaded()
    rng = np.random.default_rng(k * 1000 + m)
    coeff = rng.integers(0, 256, size=(m, k), dtype=np.uint8)
    host, dev = _rand_rows(k, ncols, k + m)
    out = alloc_rows(m, ncols, "cuda", fill=0xAB)
    GemmPlan(dev, out, coeff).run()
    torch.cuda.synchronize()
    want = GF256.gemm(coeff, host)
    assert np.array_equal(out.cpu().numpy(), want)


@pytest.mark.parametrize("vec,pf,nt", [(0, 1, False), (1, 1, False), (1, 2, False), (1, 4, False), (1, 2, True),
                                       (1, 4, True), (2, 1, False), (2, 2, False), (2, 2, True)])
def test_gemm_variants_agree(vec, pf, nt):
    _native_loaded()
    k, m, ncols = 10, 4, 300001 + 16 * vec
    rng = np.random.default_rng(7)
    coeff = rng.integers(0, 256, size=(m, k), dtype=np.uint8)
    host, dev = _rand_rows(k, ncols, 3)
    out = alloc_rows(m, ncols, "cuda", fill=0)
    GemmPlan(dev, out, coeff).run(vec=vec, pf=pf, nt=nt)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), GF256.gemm(coeff, host))


@pytest.mark.parametrize("k", [4, 8, 10, 16])
@pytest.mark.parametrize("m,pf", [(4, 0), (4, -1), (4, -2), (2, 0), (3, 0), (1, 0)])
def test_gemm_rows_in_flight_kernel(k, m, pf):
    """The rows-in-flight kernel (gf_gemm_rows_kernel: all k row loads issued before the first
    multiply, compile-time k) at every k it is built for, with its own output tile size (pf = 0) or
    1- / 2-row tiles (pf = -1 / -2), fused copies of every other input row, and a ragged tail:
    bit-exact against the oracle."""
    _native_loaded()
    ncols = 16 * 40000 + 11
    rng = np.random.default_rng(k * 100 + m)
    coeff = rng.integers(0, 256, size=(m, k), dtype=np.uint8)
    host, dev = _rand_rows(k, ncols, k + m + 5)
    out = alloc_rows(m, ncols, "cuda", fill=0)
    cdst = alloc_rows(k, ncols, "cuda", fill=0x44)
    copies = [cdst[j] if j % 2 else None for j in range(k)]
    GemmPlan(dev, out, coeff, copies=copies).run(vec=1, pf=pf, nt=True)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), GF256.gemm(coeff, host))
    c = cdst.cpu().numpy()
    for j in range(k):
        assert np.array_equal(c[j], host[j] if j % 2 else np.full(ncols, 0x44, np.uint8)), j


def test_gemm_grid_cap_and_column_window():
    _native_loaded()
    k, m, ncols = 6, 3, 200000
    coeff = np.random.default_rng(1).integers(0, 256, size=(m, k), dtype=np.uint8)
    host, dev = _rand_rows(k, ncols, 11)
    out = alloc_rows(m, ncols, "cuda", fill=0)
    plan = GemmPlan(dev, out, coeff)
    plan.run(max_blocks=3)  # the reference's -p knob: grid-stride over a capped grid
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), GF256.gemm(coeff, host))
    out.zero_()
    plan.run(col0=4096, ncols=50000)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert not got[:, :4096].any() and not got[:, 54096:].any()
    assert np.array_equal(got[:, 4096:54096], GF256.gemm(coeff, host[:, 4096:54096]))


def test_gemm_unaligned_rows_use_byte_kernel():
    _native_loaded()
    k, m, ncols = 5, 2, 10001
    coeff = np.random.default_rng(2).integers(0, 256, size=(m, k), dtype=np.uint8)
    host = np.random.default_rng(3).integers(0, 256, size=(k, ncols + 3), dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    rows = [buf[j, 3:] for j in range(k)]  # 3-byte offset: unaligned
    out = torch.zeros((m, ncols), dtype=torch.uint8, device="cuda")
    plan = GemmPlan(rows, out, coeff)
    assert plan.bytewise
    plan.run()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), GF256.gemm(coeff, host[:, 3:]))


def test_fused_copy():
    _native_loaded()
    k, ncols = 6, 99999
    host, dev = _rand_rows(k, ncols, 5)
    coeff = np.random.default_rng(9).integers(0, 256, size=(2, k), dtype=np.uint8)
    out = alloc_rows(2, ncols, "cuda", fill=0)
    dst = alloc_rows(k, ncols, "cuda", fill=0)
    copies = [dst[j] if j % 2 == 0 else None for j in range(k)]
    GemmPlan(dev, out, coeff, copies=copies).run()
    torch.cuda.synchronize()
    d = dst.cpu().numpy()
    for j in range(k):
        assert np.array_equal(d[j], host[j] if j % 2 == 0 else np.zeros(ncols, np.uint8))
    assert np.array_equal(out.cpu().numpy(), GF256.gemm(coeff, host))


def test_gf16_nibble_maps_on_device():
    _native_loaded()
    k, m, ncols = 4, 2, 50000
    f = gf.field(4)
    coeff = f.vandermonde_ref(k, m)
    maps = np.stack([np.stack([gf.byte_map_gf16_nibbles(int(coeff[i, j])) for j in range(k)]) for i in range(m)])
    host, dev = _rand_rows(k, ncols, 21)
    out = alloc_rows(m, ncols, "cuda", fill=0)
    GemmPlan(dev, out, maps=maps).run()
    torch.cuda.synchronize()
    want = np.zeros((m, ncols), np.uint8)
    for i in range(m):
        for j in range(k):
            want[i] ^= maps[i, j][host[j]]
    assert np.array_equal(out.cpu().numpy(), want)


@pytest.mark.parametrize("n", [1, 4, 10, 33, 128, 255, 256])
def test_invert_matches_oracle(n):
    _native_loaded()
    rng = np.random.default_rng(n)
    while True:
        a = rng.integers(0, 256, size=(n, n), dtype=np.uint8)
        if GF256.is_invertible(a):
            break
    inv, status = gf_invert(torch.from_numpy(a).cuda())
    assert int(status.item()) == 0
    assert np.array_equal(inv.cpu().numpy(), GF256.invert(a))


def test_invert_batch_and_singular():
    _native_loaded()
    g = GF256.generator(GF256.vandermonde_ref(10, 4))
    bad = GF256.singular_patterns(g, 10)[:3]
    good = [(0, 1, 2, 3, 4, 5, 6, 10, 11, 12), (4, 5, 6, 7, 8, 9, 10, 11, 12, 13)]
    mats = np.stack([g[list(r)] for r in good + bad])
    inv, status = gf_invert(torch.from_numpy(mats).cuda(), check=False)
    st = status.cpu().numpy()
    assert st.tolist() == [0, 0, 1, 1, 1]
    for b, rows in enumerate(good):
        assert np.array_equal(inv[b].cpu().numpy(), GF256.invert(g[list(rows)]))
    assert not inv[2:].cpu().numpy().any()
    # row pivoting: the reference's column-pivot decoder permutes output for this conf
    a = GF256.generator(GF256.vandermonde_ref(4, 2))[[2, 3, 4, 5]]
    inv, _ = gf_invert(torch.from_numpy(np.ascontiguousarray(a)).cuda())
    assert np.array_equal(GF256.matmul(a, inv.cpu().numpy()), np.eye(4, dtype=np.uint8))


def test_invert_into_plan_decodes():
    _native_loaded()
    k, p, ncols = 10, 4, 123457
    e = GF256.vandermonde_ref(k, p)
    g = GF256.generator(e)
    host, dev = _rand_rows(k, ncols, 99)
    parity = GF256.gemm(e, host)
    rows = [0, 1, 4, 5, 7, 8, 10, 11, 12, 13]  # erase natives 2, 3, 6, 9
    surv = np.stack([host[r] if r < k else parity[r - k] for r in rows])
    sdev = alloc_rows(k, ncols, "cuda")
    sdev.copy_(torch.from_numpy(surv))
    erased = [2, 3, 6, 9]
    out = alloc_rows(len(erased), ncols, "cuda", fill=0)
    plan = GemmPlan(sdev, out, device_tables=True)
    status = invert_into_plan(torch.from_numpy(g[rows].copy()).cuda(), plan, erased)
    plan.run()
    torch.cuda.synchronize()
    assert int(status.item()) == 0
    assert np.array_equal(out.cpu().numpy(), host[erased])


def test_fill_random_deterministic_and_spread():
    _native_loaded()
    a = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
    b = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
    fill_random_(a, 5)
    fill_random_(b, 5)
    assert torch.equal(a, b)
    fill_random_(b, 6)
    assert not torch.equal(a, b)
    hist = torch.bincount(a.long(), minlength=256).float()
    assert hist.min() > 0.8 * hist.mean()


@pytest.mark.parametrize("kind", ["vandermonde", "cauchy"])
def test_gen_matrix_device(kind):
    _native_loaded()
    for k, p in [(10, 4), (17, 23), (200, 56)]:
        got = gen_matrix_device(kind, k, p).cpu().numpy()
        assert np.array_equal(got, GF256.encoding_matrix(kind, k, p)), (k, p)


@pytest.mark.parametrize("engine", ["mfma", "mfma_mg2", "mfma_scattered", "mfma_i8"])
@pytest.mark.parametrize("k,m,ncols", [(128, 32, 512 * 40 + 123), (16, 4, 512 * 9), (10, 4, 512 * 7 + 5),
                                        (4, 2, 100), (32, 20, 512 * 3 + 64), (255, 1, 1024), (8, 9, 4096 + 512),
                                        (256, 40, 2048 + 2), (200, 56, 768)])
def test_mfma_bitmatrix_gemm_matches_oracle(k, m, ncols, engine):
    _native_loaded()
    rng = np.random.default_rng(k * 7 + m)
    coeff = rng.integers(0, 256, size=(m, k), dtype=np.uint8)
    host, dev = _rand_rows(k, ncols, k * m)
    out = alloc_rows(m, ncols, "cuda", fill=0x5A)
    kw = dict(engine="mfma", mfma_mg=2) if engine == "mfma_mg2" else dict(engine=engine)
    inputs = dev
    if engine == "mfma_scattered":
        # separately allocated rows in a shuffled order: the FP4 kernel's pointer-table path
        kw = dict(engine="mfma")
        order = np.random.default_rng(k).permutation(k)
        rows = [None] * k
        for j in order:
            rows[j] = dev[j].clone()
        inputs = rows
    plan = GemmPlan(inputs, out, coeff, **kw)
    if engine == "mfma_scattered" and k > 2:
        assert plan.in_stride == 0
    elif engine in ("mfma", "mfma_mg2"):
        assert plan.in_stride != 0
    plan.run()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), GF256.gemm(coeff, host))


@pytest.mark.parametrize("batch,k,m,ncols", [(3, 10, 4, 4099), (64, 4, 2, 1 << 14), (5, 16, 20, 777), (2, 1, 1, 16)])
def test_batched_gemm_matches_oracle(batch, k, m, ncols):
    _native_loaded()
    rng = np.random.default_rng(batch * 100 + k)
    coeff = rng.integers(0, 256, size=(m, k), dtype=np.uint8)
    host = rng.integers(0, 256, size=(batch, k, ncols), dtype=np.uint8)
    pitch = (ncols + 255) // 256 * 256
    dbase = torch.zeros(batch * k * pitch, dtype=torch.uint8, device="cuda")
    data = dbase.as_strided((batch, k, ncols), (k * pitch, pitch, 1))
    data.copy_(torch.from_numpy(host))
    obase = torch.full((batch * m * pitch,), 0xEE, dtype=torch.uint8, device="cuda")
    out = obase.as_strided((batch, m, ncols), (m * pitch, pitch, 1))
    plan = GemmPlan(data, out, coeff)
    assert plan.batch == batch
    plan.run()
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for b in range(batch):
        assert np.array_equal(got[b], GF256.gemm(coeff, host[b])), b


def test_auto_engine_wide_stripe_uses_matrix_cores_and_matches():
    _native_loaded()
    k, m, ncols = 96, 24, 256 * 37 + 77
    rng = np.random.default_rng(5)
    coeff = rng.integers(0, 256, size=(m, k), dtype=np.uint8)
    host, dev = _rand_rows(k, ncols, 3)
    out = alloc_rows(m, ncols, "cuda", fill=0x11)
    plan = GemmPlan(dev, out, coeff)
    assert plan.engine == "mfma"
    plan.run()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), GF256.gemm(coeff, host))
    coeff2 = rng.integers(0, 256, size=(m, k), dtype=np.uint8)
    plan.set_coeff(coeff2)  # rebuilds the bit-matrix too
    plan.run()
    plan.run(col0=1, ncols=ncols - 1)  # odd column start: v_perm fallback on the same plan
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), GF256.gemm(coeff2, host))


@pytest.mark.parametrize("k,m,ncols", [(128, 32, 256 * 41 + 99), (80, 17, 256 * 9), (255, 20, 3000)])
def test_fp4_fused_copy_and_device_coeff(k, m, ncols):
    """FP4 engine with the decode shape: scattered survivor rows, fused copies of some inputs, and
    the coefficient operand rebuilt on device from selected rows of a device matrix."""
    _native_loaded()
    rng = np.random.default_rng(k + m)
    host, dev = _rand_rows(k, ncols, k)
    rows = [dev[j].clone() for j in rng.permutation(k)]  # scattered allocations
    perm_host = np.stack([r.cpu().numpy() for r in rows])
    out = alloc_rows(m, ncols, "cuda", fill=0x33)
    cdst = alloc_rows(k, ncols, "cuda", fill=0x44)
    copies = [cdst[j] if j % 3 else None for j in range(k)]
    big = rng.integers(0, 256, size=(k, k), dtype=np.uint8)  # rows of a "device inverse"
    sel = sorted(rng.choice(k, size=m, replace=False).tolist())
    coeff = big[sel]
    plan = GemmPlan(rows, out, copies=copies, device_tables=True, engine="mfma")
    assert plan.engine == "mfma"  # (the copy variant always reads the row-pointer table)
    plan.set_coeff(coeff)  # v_perm tables (remainder columns) + bit-matrix
    plan.set_device_coeff(torch.from_numpy(big).cuda(), torch.tensor(sel, dtype=torch.int32, device="cuda"))
    plan.run()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), GF256.gemm(coeff, perm_host))
    got = cdst.cpu().numpy()
    for j in range(k):
        assert np.array_equal(got[j], perm_host[j] if j % 3 else np.full(ncols, 0x44, np.uint8)), j


@pytest.mark.parametrize("m", [26, 20, 32, 12])
def test_fp4_fused_copy_decode_shape(m):
    """The wide decode's shape: k = 128 scattered survivors, m rebuilt rows, and copies for the first
    128 - m inputs only (the surviving natives; the parity survivors have no destination). Whole
    16-row ring slots then hold no destination at all, so every wave takes the fused-copy store's
    lane-0 sink path there, and the rows around the boundary take the masked path. Bit-exact outputs
    and copies, and the copy buffers of destination-less rows stay untouched."""
    _native_loaded()
    k = 128
    ncols = 256 * (256 * 2 + 3) + 41  # several chunks per persistent block + a v_perm remainder
    rng = np.random.default_rng(1000 + m)
    host, dev = _rand_rows(k, ncols, 7 * m)
    inputs = [dev[j].clone() for j in range(k)]
    coeff = rng.integers(0, 256, size=(m, k), dtype=np.uint8)
    out = alloc_rows(m, ncols, "cuda", fill=0x5A)
    cdst = alloc_rows(k, ncols, "cuda", fill=0x44)
    ncopy = k - m
    copies = [cdst[j] if j < ncopy else None for j in range(k)]
    plan = GemmPlan(inputs, out, coeff, copies=copies, engine="mfma")
    assert plan.engine == "mfma"
    plan.run()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), GF256.gemm(coeff, host))
    got = cdst.cpu().numpy()
    assert np.array_equal(got[:ncopy], host[:ncopy])
    assert (got[ncopy:] == 0x44).all()


@pytest.mark.parametrize("k,m", [(128, 26), (128, 20), (128, 24), (120, 21), (113, 17), (128, 32), (128, 29),
                                 (116, 30)])
@pytest.mark.parametrize("variant", ["uniform", "scattered", "copy"])
@pytest.mark.parametrize("nblk", [256 * 3 + 5, 256 * 2, 40])
def test_fp4_tile_major_kernel_matches_oracle(k, m, variant, nblk, monkeypatch):
    """The tile-major FP4 kernel (gf_gemm_fp4tm_kernel, GFRS_TUNE=fp4=tm: the chunk's B resident
    in AGPRs, tiles in turn, 5..8 M-tiles; at 8 tiles tile 7's A is register-resident). Column counts give the persistent blocks an odd or an
    even number of chunks (the phantom chunk and the drain after the loop) or a single one, plus a
    v_perm remainder. The fused copy covers the first inputs only (the decode layout). Bit-exact
    against the oracle, and nothing is written outside the outputs' and copies' columns."""
    _native_loaded()
    monkeypatch.setenv("GFRS_TUNE", "fp4=tm")
    ncols = 256 * nblk + 77
    rng = np.random.default_rng(k * 131 + m * 7 + nblk)
    coeff = rng.integers(0, 256, size=(m, k), dtype=np.uint8)
    host, dev = _rand_rows(k, ncols, k + m + nblk)
    inputs, want_in = dev, host
    copies = None
    if variant in ("scattered", "copy"):
        perm = rng.permutation(k)
        inputs = [dev[j].clone() for j in perm]
        want_in = host[perm]
    ncopy = k - m
    if variant == "copy":
        cdst = alloc_rows(k, ncols, "cuda", fill=0x44)
        copies = [cdst[j] if j < ncopy else None for j in range(k)]
    out = alloc_rows(m, ncols, "cuda", fill=0x5A)
    plan = GemmPlan(inputs, out, coeff, copies=copies, engine="mfma")
    plan.run()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), GF256.gemm(coeff, want_in))
    if copies is not None:
        c = cdst.cpu().numpy()
        assert np.array_equal(c[:ncopy], want_in[:ncopy])
        assert (c[ncopy:] == 0x44).all()


@pytest.mark.parametrize("m,copy", [(26, True), (26, False), (20, False), (30, True)])
def test_fp4_tile_major_column_windows(m, copy):
    """Windowed launches on the tile-major kernel (its default shapes): three column windows with
    ragged starts and lengths, as the windowed codecs issue them, fill exactly their columns.
    Outputs and copies are bit-exact inside each window and untouched outside."""
    _native_loaded()
    k, ncols = 128, 256 * 700 + 90
    rng = np.random.default_rng(m * 17 + copy)
    coeff = rng.integers(0, 256, size=(m, k), dtype=np.uint8)
    host, dev = _rand_rows(k, ncols, 3 * m + copy)
    inputs = [dev[j].clone() for j in range(k)]
    out = alloc_rows(m, ncols, "cuda", fill=0x5A)
    cdst = alloc_rows(k, ncols, "cuda", fill=0x44) if copy else None
    copies = [cdst[j] if j < k - m else None for j in range(k)] if copy else None
    plan = GemmPlan(inputs, out, coeff, copies=copies, engine="mfma")
    windows = [(0, 256 * 100), (256 * 100 + 2, 256 * 333 + 46), (256 * 500, ncols - 256 * 500)]
    for c0, n in windows:
        plan.run(col0=c0, ncols=n)
    torch.cuda.synchronize()
    want = GF256.gemm(coeff, host)
    got = out.cpu().numpy()
    mask = np.zeros(ncols, dtype=bool)
    for c0, n in windows:
        mask[c0:c0 + n] = True
    assert np.array_equal(got[:, mask], want[:, mask])
    assert (got[:, ~mask] == 0x5A).all()
    if copy:
        c = cdst.cpu().numpy()
        assert np.array_equal(c[: k - m][:, mask], host[: k - m][:, mask])
        assert (c[: k - m][:, ~mask] == 0x44).all() and (c[k - m:] == 0x44).all()


@pytest.mark.parametrize("k,n,matrix", [(10, 14, "vandermonde"), (128, 160, "cauchy"), (4, 6, "vandermonde"),
                                        (200, 255, "sys_vandermonde")])
def test_decode_system_matches_host_decode_matrix(k, n, matrix):
    """The e x (e+k) systematic solve equals the rows of the full k x k inverse, and flags the
    reference Vandermonde's singular patterns."""
    from gpu_rscode_amd.ops import decode_system_into_plan
    from gpu_rscode_amd.models.rs import ReedSolomon
    _native_loaded()
    rs = ReedSolomon(k, n, matrix=matrix)
    g_dev = torch.from_numpy(np.ascontiguousarray(rs.G)).cuda()
    rng = np.random.default_rng(k * n)
    C = 4096
    checked = singular = 0
    for trial in range(12):
        erased_all = sorted(rng.choice(n, size=n - k, replace=False).tolist())
        rows = [r for r in range(n) if r not in erased_all]
        erased = [i for i in range(k) if i not in rows]
        if not erased:
            continue
        ins = alloc_rows(k, C, "cuda")
        outs = alloc_rows(len(erased), C, "cuda")
        plan = GemmPlan(ins, outs, device_tables=True, engine="valu")
        status = torch.zeros(1, dtype=torch.int32, device="cuda")
        decode_system_into_plan(g_dev, torch.tensor(rows, dtype=torch.int32, device="cuda"),
                                torch.tensor(erased, dtype=torch.int32, device="cuda"), plan, status=status)
        torch.cuda.synchronize()
        recoverable = GF256.is_invertible(rs.G[rows])
        assert int(status.item()) == (0 if recoverable else 1), (rows, erased)
        if not recoverable:
            singular += 1
            continue
        want = GF256.invert(rs.G[rows])[erased]
        tabs = plan.table_view().cpu().numpy()  # (k, m_pad, 8) perm records
        ref_tabs = np.transpose(perm_tables_from_coeff(want), (1, 0, 2))
        assert np.array_equal(tabs[:, : len(erased), :].view(np.uint32), ref_tabs.astype(np.uint32)), (rows, erased)
        checked += 1
    assert checked > 0


# every form the FP4 router (fp4_route, csrc/kernels/gf_mfma_fp4.hip) returns, with its shapes
_ROUTE_CASES = [(128, 8, False, "v1"), (128, 12, True, "v1"), (128, 16, False, "ar"), (128, 16, True, "ar"),
                (128, 20, False, "tm"), (128, 20, True, "tm"), (128, 24, False, "tm"), (128, 24, True, "tm"),
                (128, 26, True, "tm"), (128, 28, False, "tm"), (128, 32, False, "ar"), (128, 32, True, "tm"),
                (128, 40, False, "v1"), (100, 17, True, "v1"), (40, 32, False, "v1"),
                (128, 22, True, "tm"), (128, 12, False, "v1")]


@pytest.mark.parametrize("k,m,copy,form", _ROUTE_CASES)
@pytest.mark.parametrize("scattered", [False, True])
def test_fp4_router_every_form_matches_oracle(k, m, copy, form, scattered):
    """Every form the router can return (v1 LDS ring, A-resident, tile-major) on the shapes it is
    routed to, uniform or scattered inputs, fused copies: the plan reports the form, and outputs and
    copies are bit-exact against the oracle, with several chunks per persistent block and a v_perm
    remainder; nothing is written outside the outputs and the copy rows."""
    _native_loaded()
    ncols = 256 * (256 * 3 + 5) + 77
    rng = np.random.default_rng(k * 31 + m + 7 * copy)
    coeff = rng.integers(0, 256, size=(m, k), dtype=np.uint8)
    host, dev = _rand_rows(k, ncols, k + m)
    inputs, want_in = dev, host
    if scattered or copy:
        perm = rng.permutation(k)
        inputs = [dev[j].clone() for j in perm]
        want_in = host[perm]
    copies = None
    if copy:
        cdst = alloc_rows(k, ncols, "cuda", fill=0x44)
        copies = [cdst[j] if j % 4 else None for j in range(k)]
    out = alloc_rows(m, ncols, "cuda", fill=0x5A)
    plan = GemmPlan(inputs, out, coeff, copies=copies, engine="mfma")
    assert plan.fp4_form == form
    plan.run()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), GF256.gemm(coeff, want_in)), form
    if copies is not None:
        c = cdst.cpu().numpy()
        for j in range(k):
            assert np.array_equal(c[j], want_in[j] if j % 4 else np.full(ncols, 0x44, np.uint8)), (form, j)


@pytest.mark.parametrize("k,m,copy", [(128, 26, True), (128, 24, False), (128, 16, True), (128, 30, True)])
def test_fp4_forced_forms_agree(k, m, copy, monkeypatch):
    """GFRS_TUNE=fp4=v1 / ar / tm (the A/B override) on a shape each of them is built for: the
    three forms give identical bytes."""
    _native_loaded()
    ncols = 256 * 600 + 33
    rng = np.random.default_rng(k + m)
    coeff = rng.integers(0, 256, size=(m, k), dtype=np.uint8)
    host, dev = _rand_rows(k, ncols, 5 * m)
    inputs = [dev[j].clone() for j in range(k)]
    cdst = alloc_rows(k, ncols, "cuda", fill=0) if copy else None
    copies = [cdst[j] if j < k - m else None for j in range(k)] if copy else None
    got = {}
    for kernel in ("v1", "ar", "tm"):
        monkeypatch.setenv("GFRS_TUNE", f"fp4={kernel}")
        out = alloc_rows(m, ncols, "cuda", fill=0)
        plan = GemmPlan(inputs, out, coeff, copies=copies, engine="mfma")
        plan.run()
        torch.cuda.synchronize()
        got[kernel] = out.cpu().numpy()
        assert np.array_equal(got[kernel], GF256.gemm(coeff, host)), kernel
        if copy:
            assert np.array_equal(cdst.cpu().numpy()[: k - m], host[: k - m])


@pytest.mark.parametrize("k,m", [(128, 32), (128, 28), (128, 24), (128, 20), (127, 13), (120, 8), (113, 4), (128, 1)])
@pytest.mark.parametrize("variant", ["uniform", "scattered", "copy"])
def test_fp4_a_resident_kernel_matches_oracle(k, m, variant, monkeypatch):
    """The A-resident FP4 kernel (gf_gemm_fp4ar_kernel: A in AGPRs, accumulators in VGPRs, bias as
    the first MFMA's C operand) for every tile split it instantiates — 1..4 M-tiles per wave and one
    wave per column group, or two row halves (3 or 4 tiles each, padding tiles reading zero A) —
    with uniform / scattered / fused-copy inputs, several chunks per persistent block and a v_perm
    remainder: bit-exact against the oracle, copies included."""
    _native_loaded()
    ncols = 128 * (256 * 5 + 3) + 45
    rng = np.random.default_rng(k * 7 + m)
    coeff = rng.integers(0, 256, size=(m, k), dtype=np.uint8)
    host, dev = _rand_rows(k, ncols, k * 3 + m)
    inputs, want_in = dev, host
    copies = None
    if variant in ("scattered", "copy"):
        perm = rng.permutation(k)
        inputs = [dev[j].clone() for j in perm]
        want_in = host[perm]
    if variant == "copy":
        cdst = alloc_rows(k, ncols, "cuda", fill=0x44)
        copies = [cdst[j] if j % 3 else None for j in range(k)]
    monkeypatch.setenv("GFRS_TUNE", "fp4=ar")
    out = alloc_rows(m, ncols, "cuda", fill=0x5A)
    plan = GemmPlan(inputs, out, coeff, copies=copies, engine="mfma")
    plan.run()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), GF256.gemm(coeff, want_in))
    if copies is not None:
        c = cdst.cpu().numpy()
        for j in range(k):
            assert np.array_equal(c[j], want_in[j] if j % 3 else np.full(ncols, 0x44, np.uint8)), j


@pytest.mark.parametrize("k,m,ncols,ncopy", [(10, 4, 1000003, 0), (10, 4, 65536 + 5, 6), (128, 32, 70000, 0),
                                              (16, 20, 4096, 0), (3, 1, 15, 0), (256, 16, 33333, 0)])
def test_lds_lut_kernel_matches_oracle(k, m, ncols, ncopy):
    """The LDS nibble-table ablation (engine='lut', csrc/kernels/gf_gemm_lut.hip): tables built on
    device from the descriptor, any tile (m_pad 1..32), fused copies, the ragged tail on the byte kernel."""
    _native_loaded()
    rng = np.random.default_rng(k * 31 + m)
    coeff = rng.integers(0, 256, size=(m, k), dtype=np.uint8)
    host, dev = _rand_rows(k, ncols, k + 2 * m)
    out = alloc_rows(m, ncols, "cuda", fill=0x3C)
    copies = None
    if ncopy:
        dst = alloc_rows(k, ncols, "cuda", fill=0)
        copies = [dst[j] if j < ncopy else None for j in range(k)]
    plan = GemmPlan(dev, out, coeff, copies=copies, engine="lut")
    plan.run()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), GF256.gemm(coeff, host))
    if ncopy:
        assert np.array_equal(dst.cpu().numpy()[:ncopy], host[:ncopy])


def test_lds_lut_kernel_gf16_maps():
    _native_loaded()
    k, m, ncols = 4, 2, 100000
    f = gf.field(4)
    coeff = f.vandermonde_ref(k, m)
    maps = np.stack([np.stack([gf.byte_map_gf16_nibbles(int(coeff[i, j])) for j in range(k)]) for i in range(m)])
    host, dev = _rand_rows(k, ncols, 22)
    out = alloc_rows(m, ncols, "cuda", fill=0)
    GemmPlan(dev, out, maps=maps, engine="lut").run()
    torch.cuda.synchronize()
    want = np.zeros((m, ncols), np.uint8)
    for i in range(m):
        for j in range(k):
            want[i] ^= maps[i, j][host[j]]
    assert np.array_equal(out.cpu().numpy(), want)


_FORMS_SNIPPET = r"""
import sys
import numpy as np, torch
sys.path.insert(0, %r)
from gpu_rscode_amd.gf import GF256
from gpu_rscode_amd.models import alloc_rows
from gpu_rscode_amd.ops import GemmPlan
for k, m, C, copies in ((10, 4, 1000003, False), (10, 4, 1000003, True), (4, 2, 65536 + 5, True), (16, 3, 77777, False)):
    g = np.random.default_rng(k * 7 + m)
    host = g.integers(0, 256, size=(k, C), dtype=np.uint8)
    coeff = g.integers(0, 256, size=(m, k), dtype=np.uint8)
    dev = alloc_rows(k, C, "cuda"); dev.copy_(torch.from_numpy(host))
    out = alloc_rows(m, C, "cuda", fill=0xAB)
    cp = alloc_rows(k, C, "cuda", fill=0) if copies else None
    GemmPlan(dev, out, coeff, copies=[cp[j] for j in range(k)] if copies else None).run()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), GF256.gemm(coeff, host)), (k, m, C, copies)
    if copies:
        assert np.array_equal(cp.cpu().numpy(), host), (k, m, C)
print("FORMS-OK")
"""


@pytest.mark.parametrize("lat_groups", ["0", "1000000000"])
def test_rows_kernel_forms_match_oracle(lat_groups):
    """Both forms of the rows-in-flight kernel on the same shapes: GFRS_TUNE=rows_lat_groups=0 forces the
    throughput form (the 1 GiB headline's; small test launches otherwise take the latency form),
    10^9 the latency form (also for fused-copy decodes). Subprocess: the threshold is read once."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = with_tune(rows_lat_groups=lat_groups)
    r = subprocess.run([sys.executable, "-c", _FORMS_SNIPPET % root], capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0 and "FORMS-OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


_WIDE_BATCH_SNIPPET = r"""
import sys
import numpy as np, torch
sys.path.insert(0, %r)
from gpu_rscode_amd.gf import GF256
from gpu_rscode_amd.models import alloc_rows
from gpu_rscode_amd.ops import GemmPlan
for k, m, C, B, copies in ((128, 32, 512, 3, False), (128, 3, 8192, 2, True), (33, 5, 1000, 4, True),
                           (64, 16, 4099, 2, False), (40, 9, 70000, 2, True)):
    g = np.random.default_rng(k * 7 + m + C)
    host = g.integers(0, 256, size=(B, k, C), dtype=np.uint8)
    coeff = g.integers(0, 256, size=(m, k), dtype=np.uint8)
    ins = [alloc_rows(k, C, "cuda") for _ in range(B)]
    for b in range(B):
        ins[b].copy_(torch.from_numpy(host[b]))
    outs = [alloc_rows(m, C, "cuda", fill=0xAB) for _ in range(B)]
    cps = [alloc_rows(k, C, "cuda", fill=0) for _ in range(B)] if copies else None
    plan = GemmPlan([[r for r in x] for x in ins], [[r for r in o] for o in outs], coeff,
                    copies=[[c[j] if j %% 3 else None for j in range(k)] for c in cps] if copies else None)
    plan.run()
    torch.cuda.synchronize()
    for b in range(B):
        assert np.array_equal(outs[b].cpu().numpy(), GF256.gemm(coeff, host[b])), (k, m, C, B, b)
        if copies:
            want = host[b].copy(); want[::3] = 0
            assert np.array_equal(cps[b].cpu().numpy(), want), (k, m, C, B, b)
print("WIDE-OK")
"""


@pytest.mark.parametrize("knobs", [("0", "0"), ("0", "1000000000000"), ("1000000000000", "0")])
def test_batched_wide_kernels_match_oracle(knobs):
    """Batched wide-code launches on every kernel that can take them: the vec kernel at its widest
    tile (both knobs 0), with the tile narrowed for short rows (GFRS_TUNE short_lanes), and the k-split
    kernel (GFRS_TUNE ksplit_lanes, LDS reduction over row slices; ragged columns and fused copies
    included). Subprocess: the thresholds are read once."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = with_tune(ksplit_lanes=knobs[0], short_lanes=knobs[1])
    r = subprocess.run([sys.executable, "-c", _WIDE_BATCH_SNIPPET % root], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0 and "WIDE-OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
