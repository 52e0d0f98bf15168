"""GF(2^16) on the MI355X (csrc/kernels/gf_gemm16.hip) — bit-exact against the numpy oracle
(gpu_rscode_amd.gf.field(16)), the stand-in for an fp32 reference of an exact-integer op."""
import os
import subprocess

import numpy as np
import pytest
import torch

from gpu_rscode_amd import ReedSolomon, alloc_rows, gf
from gpu_rscode_amd.ops import Gemm16Plan
from gpu_rscode_amd.utils import fileformat as ff

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
F = gf.field(16)


def _rand(rows, C, seed):
    return torch.from_numpy(np.random.default_rng(seed).integers(0, 256, size=(rows, C), dtype=np.uint8))


def _oracle(coeff, data_u8):
    return F.gemm(coeff, np.ascontiguousarray(data_u8).view("<u2"))


@pytest.mark.parametrize("k,m,C", [(10, 4, 2 * 100_005), (4, 2, 34), (7, 3, 16 * 1000), (16, 16, 2 * 4099),
                                   (10, 24, 2 * 5003)])
def test_gemm16_matches_oracle(k, m, C):
    """Aligned rows: the 16-byte vector kernel plus the ragged tail symbols (C % 16 != 0), output tiles
    of 1..8 rows (m = 24: m_pad 32, four tiles of 8)."""
    rng = np.random.default_rng(k * 1000 + m)
    coeff = rng.integers(0, 65536, size=(m, k))
    coeff[0, :2] = [0, 1]
    x = alloc_rows(k, C, "cuda")
    x.copy_(_rand(k, C, C))
    y = alloc_rows(m, C, "cuda", fill=0xAB)
    Gemm16Plan(x, y, coeff).run()
    torch.cuda.synchronize()
    assert np.array_equal(y.cpu().numpy().view("<u2"), _oracle(coeff, x.cpu().numpy()))


@pytest.mark.parametrize("extra_groups,tail", [(100, 5), (300, 7), (256, 7), (511, 1), (0, 3)])
@pytest.mark.parametrize("m,B", [(4, 1), (2, 2), (1, 1)])
def test_gemm16_two_groups_per_lane(extra_groups, tail, m, B):
    """Long rows (>= 32768 16-byte groups) run the vector kernel with two groups per lane, 256
    groups apart. The last block's second group is live for some lanes only, and the ragged tail
    symbols land on the first or the second group slot (extra_groups < 256 or >= 256). Fused copies
    and a batch of stripes run through the same kernel. Bit-exact against the oracle, and
    destination-less rows and columns are left untouched."""
    k = 6
    C = 16 * (512 * 70 + extra_groups) + 2 * tail
    rng = np.random.default_rng(extra_groups * 31 + tail + 7 * m + B)
    coeff = rng.integers(0, 65536, size=(m, k))
    if B == 1:
        x = alloc_rows(k, C, "cuda")
        x.copy_(_rand(k, C, C + m))
        y = alloc_rows(m, C, "cuda", fill=0xAB)
        z = alloc_rows(k, C, "cuda", fill=0x44)
        copies = [z[j] if j % 2 else None for j in range(k)]
        Gemm16Plan(x, y, coeff, copies=copies, engine="valu16").run()
        torch.cuda.synchronize()
        xh = x.cpu().numpy()
        assert np.array_equal(y.cpu().numpy().view("<u2"), _oracle(coeff, xh))
        zh = z.cpu().numpy()
        for j in range(k):
            assert np.array_equal(zh[j], xh[j] if j % 2 else np.full(C, 0x44, np.uint8)), j
    else:
        x = _rand(B * k, C, C + m).view(B, k, C).cuda()
        y = torch.zeros((B, m, C), dtype=torch.uint8, device="cuda")
        Gemm16Plan(x, y, coeff, engine="valu16").run()
        torch.cuda.synchronize()
        xh, yh = x.cpu().numpy(), y.cpu().numpy()
        for b in range(B):
            assert np.array_equal(yh[b].view("<u2"), _oracle(coeff, xh[b])), b


def test_gemm16_unaligned_rows_and_column_ranges():
    """Rows 2 bytes off a 16-byte boundary take the symbol kernel; a sub-range [col0, col0 + n) only
    writes those columns."""
    k, m, C = 6, 3, 2 * 3001
    coeff = np.random.default_rng(5).integers(0, 65536, size=(m, k))
    flat = torch.zeros(k * C + 2, dtype=torch.uint8, device="cuda")
    x = flat[2:].view(k, C)
    x.copy_(_rand(k, C, 9))
    y = torch.zeros((m, C), dtype=torch.uint8, device="cuda")
    plan = Gemm16Plan([x[j] for j in range(k)], y, coeff)
    assert plan.symwise
    plan.run()
    torch.cuda.synchronize()
    want = _oracle(coeff, x.cpu().numpy())
    assert np.array_equal(y.cpu().numpy().view("<u2"), want)
    xa = alloc_rows(k, C, "cuda")
    xa.copy_(x)
    ya = alloc_rows(m, C, "cuda", fill=0)
    pa = Gemm16Plan(xa, ya, coeff)
    pa.run(col0=32, ncols=2 * 1000)  # vector kernel from an aligned start
    pa.run(col0=2 * 1017, ncols=2 * 100)  # symbol kernel from an unaligned start
    torch.cuda.synchronize()
    got = ya.cpu().numpy().view("<u2")
    assert np.array_equal(got[:, 16:16 + 1000], want[:, 16:16 + 1000])
    assert np.array_equal(got[:, 1017:1117], want[:, 1017:1117])
    assert not got[:, :16].any() and not got[:, 1117:].any() and not got[:, 1016].any()
    with pytest.raises(ValueError):
        pa.run(col0=1, ncols=2)


@pytest.mark.parametrize("k,n,C", [(10, 14, 2 * 65_539), (300, 340, 2 * 20_011)])
def test_codec_gpu_encode_decode_bit_exact(k, n, C):
    """The ReedSolomon codec in GF(2^16) on the GPU: parity equals the oracle, and decoding after
    n - k random erasures (natives and parity) rebuilds the natives with the survivors copied in the
    same pass. (300, 340) is past GF(2^8)'s n <= 256."""
    rs = ReedSolomon(k, n, field="gf65536", matrix="cauchy")
    data = alloc_rows(k, C, "cuda")
    data.copy_(_rand(k, C, n))
    par = rs.encode(data)
    torch.cuda.synchronize()
    assert np.array_equal(par.cpu().numpy().view("<u2"), _oracle(rs.E, data.cpu().numpy()))
    rng = np.random.default_rng(7)
    erased = set(rng.choice(n, size=n - k, replace=False).tolist())
    rows = [r for r in range(n) if r not in erased]
    stripe = [data[r] if r < k else par[r - k] for r in rows]
    out = alloc_rows(k, C, "cuda", fill=0)
    rs.decode(stripe, rows, out=out)
    torch.cuda.synchronize()
    assert torch.equal(out, data)


def test_gpu_cli_w16_roundtrip(tmp_path):
    """bin/RS -w 16: the streaming pipeline with GF(2^16) slices, versioned METADATA, decode reads
    the field from it."""
    size = 3_000_017
    payload = np.random.default_rng(3).integers(0, 256, size, dtype=np.uint8).tobytes()
    (tmp_path / "f.bin").write_bytes(payload)
    rs_bin = os.path.join(ROOT, "bin", "RS")
    r = subprocess.run([rs_bin, "-q", "-k", "10", "-n", "14", "-w", "16", "-s", "2", "-e", "f.bin"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr
    md = ff.read_metadata(str(tmp_path / "f.bin.METADATA"))
    assert md.w == 16
    C = ff.chunk_size(size, 10, 16)
    data = np.frombuffer(payload + bytes(10 * C - size), dtype=np.uint8).reshape(10, C)
    par = np.stack([np.frombuffer((tmp_path / f"_{10 + i}_f.bin").read_bytes(), dtype=np.uint8) for i in range(4)])
    assert np.array_equal(par.view("<u2"), F.gemm(md.e, data.view("<u2")))
    ff.write_conf(str(tmp_path / "conf"), ff.worst_case_conf("f.bin", 14, 10))
    r = subprocess.run([rs_bin, "-q", "-d", "-i", "f.bin", "-c", "conf", "-o", "o.bin"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "o.bin").read_bytes() == payload


@pytest.mark.parametrize("k,n,e,matrix", [(10, 14, 4, "vandermonde"), (300, 340, 40, "cauchy"), (6, 9, 1, "cauchy")])
def test_device_built_w16_decode_plans(k, n, e, matrix):
    """GF(2^16) PatternDecoder: the survivor list lives on the device, the kernel (gf_decode16.hip)
    checks it, derives the erased natives, solves the e x (e + k) system and writes the plan's
    tables and row pointers; the decode rebuilds the natives bit-exactly, survivors copied in the
    same pass, for several patterns through one decoder."""
    from gpu_rscode_amd.ops import PatternDecoder

    C = 2 * 9_001
    rs = ReedSolomon(k, n, field="gf65536", matrix=matrix)
    data = alloc_rows(k, C, "cuda")
    data.copy_(_rand(k, C, k + e))
    par = rs.encode(data)
    g = torch.from_numpy(np.ascontiguousarray(rs.G, dtype="<u2").view(np.int16)).cuda()
    out = alloc_rows(k, C, "cuda")
    dec = PatternDecoder(g, [data[i] for i in range(k)] + [par[i] for i in range(n - k)], [out[i] for i in range(k)], e)
    rng = np.random.default_rng(e)
    done = 0
    while done < 3:
        erased = sorted(rng.choice(k, size=e, replace=False).tolist())
        lost_par = sorted(rng.choice(n - k, size=n - k - e, replace=False).tolist())
        rows = [r for r in range(n) if r not in erased and (r < k or (r - k) not in lost_par)]
        rng.shuffle(rows)
        if not rs.is_recoverable(rows):
            continue
        out.fill_(0)
        dec.rows.copy_(torch.tensor(rows, dtype=torch.int32))
        dec.solve()
        dec.run()
        torch.cuda.synchronize()
        assert int(dec.status.item()) == 0
        assert dec.erased.tolist() == erased
        assert torch.equal(out, data), (rows, erased)
        done += 1
    # a chunk listed twice: status 2, nothing written (no output pointers)
    bad = list(range(k - 1)) + [0]
    dec.rows.copy_(torch.tensor(bad, dtype=torch.int32))
    out.fill_(7)
    dec.solve()
    dec.run()
    torch.cuda.synchronize()
    assert int(dec.status.item()) == 2 and bool((out == 7).all())


def test_rs_decode_device_invert_w16_matches_host_plan():
    """ReedSolomon.decode(device_invert=True) for GF(2^16): the device-solved plan equals the host
    one; a singular pattern reports status 1."""
    k, n, C = 12, 16, 2 * 5_003
    rs = ReedSolomon(k, n, field="gf65536")
    data = alloc_rows(k, C, "cuda")
    data.copy_(_rand(k, C, 77))
    par = rs.encode(data)
    stripe = [data[i] for i in range(k)] + [par[i] for i in range(n - k)]
    rows = [1, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 15]
    for dev_inv in (False, True):
        out = rs.decode([stripe[r] for r in rows], rows, device_invert=dev_inv)
        torch.cuda.synchronize()
        assert torch.equal(out, data), dev_inv
    assert int(rs.last_status.item()) == 0
    rs.G = np.array(rs.G)
    rs.G[14] = rs.G[12]  # two equal parity rows: any pattern using both is singular
    rows = [2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 14]
    rs.decode([stripe[r] for r in rows], rows, device_invert=True)
    torch.cuda.synchronize()
    assert int(rs.last_status.item()) == 1


@pytest.mark.parametrize("k,m,C,col", [(300, 40, 2 * 256 * 37 + 2 * 13, (0, None)), (64, 16, 512 * 9, (0, None)),
                                       (17, 20, 512 * 3 + 6, (4, 1536)), (300, 40, 512 * 5, (512, 1024)),
                                       (300, 35, 2 * 20_011, (0, None)), (150, 35, 1024 * 40, (1024, 1024 * 37 + 6))])
def test_gemm16_fp4_engine_matches_oracle(k, m, C, col):
    """GF(2^16) on the FP4 matrix cores (gf_mfma16.hip): the 16 x 16 bit-matrix of every coefficient,
    K split into passes (k = 300: later passes XOR into the outputs), 1 KiB chunks on the matrix
    cores (the ragged tail as a partial chunk); column sub-ranges write only those columns. m = 35
    takes one M-tile per block (MG = 1), whose epilogue follows its last MFMA closely."""
    rng = np.random.default_rng(k + m + C)
    coeff = rng.integers(0, 65536, size=(m, k))
    coeff[0, :3] = [0, 1, 65535]
    x = alloc_rows(k, C, "cuda")
    x.copy_(_rand(k, C, C + 1))
    y = alloc_rows(m, C, "cuda", fill=0x5A)
    plan = Gemm16Plan(x, y, coeff, engine="mfma")
    assert plan.engine == "mfma"
    c0, n = col[0], (C - col[0] if col[1] is None else col[1])
    plan.run(col0=c0, ncols=n)
    torch.cuda.synchronize()
    want = _oracle(coeff, x.cpu().numpy())
    got = y.cpu().numpy().view("<u2")
    s0, s1 = c0 // 2, (c0 + n) // 2
    assert np.array_equal(got[:, s0:s1], want[:, s0:s1])
    assert (got[:, :s0] == 0x5A5A).all() and (got[:, s1:] == 0x5A5A).all()


def test_gemm16_fp4_fused_copies_and_device_decoder():
    """The matrix-core w = 16 decode: survivors copied in the same pass (K-steps spread over the groups, every pass
    its own rows), and a PatternDecoder whose plan (tables, row pointers AND bit-matrix) is built
    on the device from the survivor list (k = 300, 40 erasures)."""
    from gpu_rscode_amd.ops import PatternDecoder

    k, n, C = 300, 340, 512 * 11 + 2 * 7
    rs = ReedSolomon(k, n, field="gf65536", matrix="cauchy")
    data = alloc_rows(k, C, "cuda")
    data.copy_(_rand(k, C, 5))
    par = rs.encode(data)
    torch.cuda.synchronize()
    assert np.array_equal(par.cpu().numpy().view("<u2"), _oracle(rs.E, data.cpu().numpy()))
    g = torch.from_numpy(np.ascontiguousarray(rs.G, dtype="<u2").view(np.int16)).cuda()
    out = alloc_rows(k, C, "cuda")
    dec = PatternDecoder(g, [data[i] for i in range(k)] + [par[i] for i in range(n - k)], [out[i] for i in range(k)],
                         40, engine="mfma")
    assert dec.engine == "mfma"
    rng = np.random.default_rng(3)
    for _ in range(2):
        erased = sorted(rng.choice(k, size=40, replace=False).tolist())
        rows = [r for r in range(k) if r not in erased] + list(range(k, n))
        rng.shuffle(rows)
        out.fill_(0)
        dec.rows.copy_(torch.tensor(rows, dtype=torch.int32))
        dec.solve()
        dec.run()
        torch.cuda.synchronize()
        assert int(dec.status.item()) == 0 and dec.erased.tolist() == erased
        assert torch.equal(out, data)


@pytest.mark.parametrize("engine_env", ["0", "1"])
@pytest.mark.parametrize("k,n,C,B", [(300, 340, 1024 * 3 + 208, 5), (64, 80, 1024 * 3, 9), (16, 20, 2 * 333, 17)])
def test_batched_w16_encode_decode(k, n, C, B, engine_env, monkeypatch):
    """GF(2^16) batched launches (ReedSolomon.encode_batch / decode_batch): B stripes in one call,
    on the matrix cores (stripes at fixed strides; every stripe's ragged rest on the batched v_perm
    kernel) and on the batched v_perm kernel alone; decode copies the survivors in the same pass."""
    monkeypatch.setenv("GFRS_TUNE", f"gf16_mfma={engine_env}")
    rs = ReedSolomon(k, n, field="gf65536", matrix="cauchy")
    data = torch.stack([_rand(k, C, 100 + b) for b in range(B)]).cuda()
    par = rs.encode_batch(data)
    torch.cuda.synchronize()
    d_host = data.cpu().numpy()
    for b in (0, B // 2, B - 1):
        assert np.array_equal(par[b].cpu().numpy().view("<u2"), _oracle(rs.E, d_host[b]))
    rng = np.random.default_rng(k + B)
    erased = sorted(rng.choice(k, size=min(n - k, k), replace=False).tolist())
    rows = [r for r in range(n) if r not in set(erased)][:k]
    surv = torch.stack([torch.stack([data[b, r] if r < k else par[b, r - k] for r in rows]) for b in range(B)])
    out = rs.decode_batch(surv, rows)
    torch.cuda.synchronize()
    assert torch.equal(out, data)


def test_batched_w16_scattered_stripes_fall_back_to_vperm():
    """Stripes that are not at fixed strides cannot take the batched matrix-core launch: the plan
    keeps the per-stripe pointer tables of the batched v_perm kernel."""
    k, m, C, B = 64, 16, 2048, 4
    rng = np.random.default_rng(4)
    coeff = rng.integers(0, 65536, size=(m, k))
    ins = [[alloc_rows(k, C, "cuda")[j] for j in range(k)] for _ in range(B)]  # separate allocations
    for st in ins:
        for r in st:
            r.copy_(torch.from_numpy(rng.integers(0, 256, C, dtype=np.uint8)))
    outs = [[alloc_rows(m, C, "cuda", fill=0)[i] for i in range(m)] for _ in range(B)]
    plan = Gemm16Plan(ins, outs, coeff)
    assert plan.batch == B and plan.in_bstride is None and plan.engine == "valu16"
    plan.run()
    torch.cuda.synchronize()
    for b in range(B):
        x = torch.stack(ins[b]).cpu().numpy()
        assert np.array_equal(torch.stack(outs[b]).cpu().numpy().view("<u2"), _oracle(coeff, x))


def _w16_setup(k, n, matrix="cauchy"):
    rs = ReedSolomon(k, n, field="gf65536", matrix=matrix)
    g = torch.from_numpy(np.ascontiguousarray(rs.G, dtype="<u2").view(np.int16)).cuda()
    return rs, g


def _solve16(g, rows, e, k, force_blocked):
    from gpu_rscode_amd.ops.gemm import Gemm16Plan
    from gpu_rscode_amd.ops.inverse import decode_system16_into_plan

    ins = alloc_rows(k, 64, "cuda")
    outs = alloc_rows(e, 64, "cuda")
    plan = Gemm16Plan(ins, outs, device_tables=True, engine="valu16")
    erased = torch.zeros(e, dtype=torch.int32, device="cuda")
    dm = torch.zeros((e, k), dtype=torch.int16, device="cuda")
    st = decode_system16_into_plan(g, torch.tensor(rows, dtype=torch.int32, device="cuda"), erased, plan, dm=dm,
                                   force_blocked=force_blocked)
    torch.cuda.synchronize()
    return int(st.item()), erased.tolist(), dm.cpu().numpy().view(np.uint16)


@pytest.mark.parametrize("k,n,e", [(10, 14, 4), (64, 100, 33), (300, 340, 40), (40, 120, 37)])
def test_blocked_w16_solve_equals_one_workgroup_solve(k, n, e):
    """The blocked multi-workgroup GF(2^16) solve (panels of pivot columns, rank-P updates over the
    chip) forced on systems the one-workgroup kernel also solves: identical decode rows, erased
    natives and status, for several random patterns (panels of 32: one, two and a ragged last)."""
    rs, g = _w16_setup(k, n)
    rng = np.random.default_rng(k * 7 + e)
    for _ in range(3):
        erased = sorted(rng.choice(k, size=e, replace=False).tolist())
        par = sorted(rng.choice(range(k, n), size=e, replace=False).tolist())
        rows = [r for r in range(k) if r not in erased] + par
        rng.shuffle(rows)
        one = _solve16(g, rows, e, k, False)
        blk = _solve16(g, rows, e, k, True)
        assert one[0] == blk[0] == 0
        assert one[1] == blk[1] == erased
        assert np.array_equal(one[2], blk[2])
        assert np.array_equal(blk[2], rs._erased_rows(rows, erased))


def test_blocked_w16_solve_flags_singular_and_invalid_patterns():
    k, n, e = 20, 30, 6
    rs, _ = _w16_setup(k, n)
    G = np.array(rs.G)
    G[k + 3] = G[k + 1]  # two equal parity rows: any pattern using both is singular
    g = torch.from_numpy(np.ascontiguousarray(G, dtype="<u2").view(np.int16)).cuda()
    rows = list(range(e, k)) + [k + 1, k + 3, k + 4, k + 5, k + 6, k + 7]
    assert _solve16(g, rows, e, k, True)[0] == 1
    bad = list(range(k - 1)) + [0]  # a chunk listed twice
    assert _solve16(g, bad, 1, k, True)[0] == 2


@pytest.mark.parametrize("k,n,e", [(2000, 2100, 100), (600, 1000, 300)])
def test_blocked_w16_decode_large_systems_end_to_end(k, n, e):
    """Systems past one workgroup: k = 2000 with e = 100 (the e x (e + k) system is 420 KB) and
    e = 300 > 256. PatternDecoder builds the plan on the device (blocked solve) and the decode
    rebuilds every erased native bit-exactly; the decode rows equal the host solve's
    (gfrs::gf16w::decode_rows)."""
    from gpu_rscode_amd.ops import PatternDecoder

    C = 2 * 1024 + 32
    rs, g = _w16_setup(k, n, "cauchy")
    assert not __import__("gpu_rscode_amd")._native.hip().decode_system16_supported(n, k, e)
    data = alloc_rows(k, C, "cuda")
    data.copy_(_rand(k, C, 3 + e))
    par = rs.encode(data)
    out = alloc_rows(k, C, "cuda")
    dec = PatternDecoder(g, [data[i] for i in range(k)] + [par[i] for i in range(n - k)], [out[i] for i in range(k)], e)
    rng = np.random.default_rng(k + e)
    erased = sorted(rng.choice(k, size=e, replace=False).tolist())
    rows = [r for r in range(k) if r not in erased] + sorted(rng.choice(range(k, n), size=e, replace=False).tolist())
    rng.shuffle(rows)
    dec.rows.copy_(torch.tensor(rows, dtype=torch.int32))
    dec.solve()
    dec.run()
    torch.cuda.synchronize()
    assert int(dec.status.item()) == 0
    assert dec.erased.tolist() == erased
    assert torch.equal(out, data)
    dm = torch.zeros((e, k), dtype=torch.int16, device="cuda")
    from gpu_rscode_amd.ops.inverse import decode_system16_into_plan
    decode_system16_into_plan(g, torch.tensor(rows, dtype=torch.int32, device="cuda"), dec.erased, dec.plan,
                              ptrs=dec.ptrs, dm=dm)
    torch.cuda.synchronize()
    assert np.array_equal(dm.cpu().numpy().view(np.uint16), rs._erased_rows(rows, erased))
