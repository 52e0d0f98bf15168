"""End-to-end codec on the GPU: ReedSolomon model, host streaming pipeline, file codec, bin/RS."""
import itertools
import os
import subprocess

import numpy as np
import pytest
import torch

from gpu_rscode_amd import ReedSolomon, alloc_rows
from gpu_rscode_amd.gf import GF256
from gpu_rscode_amd._build import binary
from gpu_rscode_amd._native import cpu, hip
from gpu_rscode_amd.utils import fileformat as ff

pytestmark = pytest.mark.gpu


def _data(k, C, seed=0):
    host = np.random.default_rng(seed).integers(0, 256, size=(k, C), dtype=np.uint8)
    dev = alloc_rows(k, C, "cuda")
    dev.copy_(torch.from_numpy(host))
    return host, dev


@pytest.mark.parametrize("matrix", ["vandermonde", "cauchy", "sys_vandermonde"])
def test_all_erasure_subsets_k4_n6(matrix):
    rs = ReedSolomon(4, 6, matrix=matrix)
    host, data = _data(4, 65537)
    parity = rs.encode(data)
    stripe = [data[i] for i in range(4)] + [parity[i] for i in range(2)]
    for rows in itertools.combinations(range(6), 4):
        for dev_inv in (False, True):
            out = rs.decode([stripe[r] for r in rows], rows, device_invert=dev_inv)
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy(), host), (rows, dev_inv)


def test_k10_n14_odd_chunk_random_patterns():
    k, n = 10, 14
    rs = ReedSolomon(k, n)
    C = 1_000_003
    host, data = _data(k, C, 1)
    parity = rs.encode(data)
    torch.cuda.synchronize()
    assert np.array_equal(parity.cpu().numpy(), GF256.gemm(rs.E, host))
    stripe = [data[i] for i in range(k)] + [parity[i] for i in range(n - k)]
    rng = np.random.default_rng(2)
    tested = 0
    while tested < 12:
        erased = set(rng.choice(n, size=4, replace=False).tolist())
        rows = [r for r in range(n) if r not in erased]
        if not rs.is_recoverable(rows):
            continue
        out = rs.decode([stripe[r] for r in rows], rows, device_invert=bool(tested % 2))
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), host), sorted(erased)
        tested += 1


def test_device_invert_flags_singular_pattern():
    rs = ReedSolomon(10, 14)
    host, data = _data(10, 4096)
    parity = rs.encode(data)
    stripe = [data[i] for i in range(10)] + [parity[i] for i in range(4)]
    bad = GF256.singular_patterns(rs.G, 10)[0]
    rs.decode([stripe[r] for r in bad], bad, device_invert=True)
    torch.cuda.synchronize()
    assert int(rs.last_status.item()) == 1


def test_reassigning_g_drops_cached_decode_plans():
    """Decode a pattern, replace E and G by another code's, re-encode and decode the SAME pattern on
    the SAME buffers: the cached plan (keyed on buffers + pattern) must not replay the old inverse."""
    k, n = 8, 11
    rs = ReedSolomon(k, n)
    other = ReedSolomon(k, n, matrix="cauchy")
    host, data = _data(k, 20_011, 6)
    parity = alloc_rows(n - k, 20_011, "cuda")
    out = alloc_rows(k, 20_011, "cuda")
    rows = [2, 3, 4, 5, 6, 7, 8, 9]  # natives 0, 1 lost
    for code in (rs, other):
        if code is other:
            rs.E, rs.G = other.E, other.G
        rs.encode(data, parity)
        stripe = [data[i] for i in range(k)] + [parity[i] for i in range(n - k)]
        rs.decode([stripe[r] for r in rows], rows, out=out)
        torch.cuda.synchronize()
        assert np.array_equal(parity.cpu().numpy(), GF256.gemm(other.E if code is other else rs.E, host))
        assert np.array_equal(out.cpu().numpy(), host)


def test_reconstruct_natives_and_parity_in_place():
    k, n = 12, 16
    rs = ReedSolomon(k, n, matrix="cauchy")
    C = 300_001
    host, data = _data(k, C, 3)
    stripe = alloc_rows(n, C, "cuda")
    stripe[:k].copy_(data)
    rs.encode([stripe[i] for i in range(k)], [stripe[i] for i in range(k, n)])
    want = stripe.clone()
    erased = [0, 5, 13, 15]
    stripe[erased] = 0
    rs.reconstruct(stripe, erased)
    torch.cuda.synchronize()
    assert torch.equal(stripe, want)


def test_gf16_field_on_gpu():
    rs = ReedSolomon(6, 9, field="gf16")
    host, data = _data(6, 10007, 4)
    parity = rs.encode(data)
    stripe = [data[i] for i in range(6)] + [parity[i] for i in range(3)]
    cpu_par = rs.encode(torch.from_numpy(host))
    assert np.array_equal(parity.cpu().numpy(), cpu_par.numpy())
    for rows in [(3, 4, 5, 6, 7, 8), (0, 2, 4, 6, 7, 8)]:
        out = rs.decode([stripe[r] for r in rows], rows)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), host)


def test_wide_stripe_k128_n160():
    k, n = 128, 160
    rs = ReedSolomon(k, n, matrix="cauchy")
    C = 40_003
    host, data = _data(k, C, 5)
    parity = rs.encode(data)
    torch.cuda.synchronize()
    assert np.array_equal(parity.cpu().numpy(), GF256.gemm(rs.E, host))
    stripe = [data[i] for i in range(k)] + [parity[i] for i in range(n - k)]
    rows = list(range(32, 160))  # lose the first 32 natives
    out = rs.decode([stripe[r] for r in rows], rows, device_invert=True)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), host)
    # mixed erasures (natives + parity), host-inverted: FP4 engine with fused survivor copies
    erased = set(range(0, 128, 7)) | {130, 141, 150}
    rows = [r for r in range(160) if r not in erased][:128]
    for dev_inv in (False, True):
        out = rs.decode([stripe[r] for r in rows], rows, device_invert=dev_inv)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), host), dev_inv


@pytest.mark.parametrize("streams,slice_", [(1, 1 << 20), (2, 1 << 20), (4, 3 << 18), (3, 256)])
def test_host_pipeline_streams(streams, slice_):
    k, p, C = 10, 4, 3_000_017
    rng = np.random.default_rng(streams)
    host = torch.from_numpy(rng.integers(0, 256, size=(k, C), dtype=np.uint8)).pin_memory()
    par = torch.zeros((p, C), dtype=torch.uint8).pin_memory()
    e = GF256.vandermonde_ref(k, p)
    res = hip().gemm_host([0], [host[j].data_ptr() for j in range(k)], [par[i].data_ptr() for i in range(p)],
                          e.tobytes(), C, streams, slice_, 0, False)
    assert res["devices"][0]["bytes_h2d"] == k * C
    assert np.array_equal(par.numpy(), GF256.gemm(e, host.numpy()))


def test_host_pipeline_workspace_reuse_across_shapes_and_coefficients():
    rng = np.random.default_rng(77)
    h = hip()
    for k, p, C in [(10, 4, 1_000_003), (10, 4, 1_000_003), (16, 8, 3_000_001), (4, 2, 999), (16, 8, 3_000_001)]:
        host = torch.from_numpy(rng.integers(0, 256, size=(k, C), dtype=np.uint8)).pin_memory()
        par = torch.zeros((p, C), dtype=torch.uint8).pin_memory()
        e = rng.integers(0, 256, size=(p, k), dtype=np.uint8)  # a new matrix every call
        h.gemm_host([0], [host[j].data_ptr() for j in range(k)], [par[i].data_ptr() for i in range(p)],
                    e.tobytes(), C, 3, 1 << 18, 0, False)
        assert np.array_equal(par.numpy(), GF256.gemm(e, host.numpy())), (k, p, C)
    h.release_workspaces()


def test_file_codec_gpu_and_cross_compat_with_cpu(tmp_path):
    f = tmp_path / "f.bin"
    payload = os.urandom(2_000_003)
    f.write_bytes(payload)
    hip().encode_file(str(f), 10, 4, "vandermonde", False, [0], 2, 1 << 20, 0)
    parity_gpu = [(tmp_path / f"_{i}_f.bin").read_bytes() for i in range(14)]
    g2 = tmp_path / "g"
    g2.mkdir()
    (g2 / "f.bin").write_bytes(payload)
    cpu().encode_file(str(g2 / "f.bin"), 10, 4)
    assert parity_gpu == [(g2 / f"_{i}_f.bin").read_bytes() for i in range(14)]
    conf = tmp_path / "conf"
    ff.write_conf(str(conf), [ff.chunk_path(str(f), r) for r in (0, 2, 3, 5, 6, 8, 10, 11, 12, 13)])
    hip().decode_file(str(f), str(conf), str(tmp_path / "o_gpu"), [0], 3, 1 << 19, 0)
    cpu().decode_file(str(f), str(conf), str(tmp_path / "o_cpu"))
    assert (tmp_path / "o_gpu").read_bytes() == payload == (tmp_path / "o_cpu").read_bytes()


def test_rs_cli_reference_flags(tmp_path):
    exe = str(binary("RS"))
    payload = os.urandom(3_333_333)
    (tmp_path / "f.bin").write_bytes(payload)
    r = subprocess.run([exe, "-k", "4", "-n", "6", "-e", "f.bin", "-s", "2", "-p", "64"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Total GPU encoding time" in r.stdout
    subprocess.run([exe, "-k", "4", "-n", "6", "-e", "f.bin", "--make-conf"], cwd=tmp_path, check=True,
                   capture_output=True, timeout=60)
    r = subprocess.run([exe, "-d", "-i", "f.bin", "-c", "conf-6-4-f.bin", "-o", "out.bin", "-s", "4"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "out.bin").read_bytes() == payload


def test_batched_encode_decode_small_objects():
    k, n, B, C = 10, 14, 256, 40_001
    rs = ReedSolomon(k, n)
    host = np.random.default_rng(9).integers(0, 256, size=(B, k, C), dtype=np.uint8)
    data = torch.from_numpy(host).cuda()
    parity = rs.encode_batch(data)
    torch.cuda.synchronize()
    for b in (0, 77, B - 1):
        assert np.array_equal(parity[b].cpu().numpy(), GF256.gemm(rs.E, host[b]))
    rows = [0, 2, 3, 4, 6, 7, 9, 10, 11, 13]  # natives 1, 5, 8 lost on every stripe
    stripe = torch.cat([data, parity], dim=1)
    out = rs.decode_batch(stripe[:, rows].contiguous(), rows)
    torch.cuda.synchronize()
    assert torch.equal(out, data)


def test_batched_plans_survive_many_per_object_plans_into_a_graph_capture():
    """A captured hipGraph of encode_batch / decode_batch must find their cached plans even after
    more than 64 other plans were built (per-object encodes): a miss during capture would build a
    plan, whose descriptor upload a capturing stream refuses (scripts/serve_bench.py hit this)."""
    k, n, B, C = 10, 14, 70, 8_192
    rs = ReedSolomon(k, n)
    host = np.random.default_rng(4).integers(0, 256, size=(B, k, C), dtype=np.uint8)
    data = torch.from_numpy(host).cuda()
    parity = torch.empty((B, n - k, C), dtype=torch.uint8, device="cuda")
    rows = [0, 2, 3, 4, 6, 7, 9, 10, 11, 13]
    surv = torch.empty((B, k, C), dtype=torch.uint8, device="cuda")
    out = torch.empty((B, k, C), dtype=torch.uint8, device="cuda")
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        rs.encode_batch(data, parity)
        for j, r in enumerate(rows):
            surv[:, j].copy_(data[:, r] if r < k else parity[:, r - k])
        rs.decode_batch(surv, rows, out)
        for b in range(B):  # 70 per-object plans on top of the two batched ones
            rs.encode(data[b], parity[b])
    torch.cuda.synchronize()
    parity.zero_()
    out.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        rs.encode_batch(data, parity)
        rs.decode_batch(surv, rows, out)
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(parity[B - 1].cpu().numpy(), GF256.gemm(rs.E, host[B - 1]))
    assert torch.equal(out, data)


def test_cached_plans_do_not_pin_the_callers_buffers():
    """Encoding / decoding fresh buffers in a loop must not keep the old ones allocated: the plan
    cache keys plans by row pointers and its plans hold no tensor references (a cache that pinned
    its buffers would keep up to 512 generations of 1-GiB stripes alive)."""
    k, n, C = 10, 14, 1 << 20
    rs = ReedSolomon(k, n)
    rows = [0, 1, 2, 5, 6, 8, 10, 11, 12, 13]
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    for it in range(12):
        data = alloc_rows(k, C, "cuda", fill=it)
        parity = rs.encode(data)
        par2 = alloc_rows(n - k, C, "cuda")
        rs.encode(data, par2)  # the 2-D fast-path key
        stripe = [data[i] for i in range(k)] + [parity[i] for i in range(n - k)]
        out = rs.decode([stripe[r] for r in rows], rows)
        out2 = rs.decode([stripe[r] for r in rows], rows, device_invert=True)
        batch = rs.encode_batch(data.unsqueeze(0))
        torch.cuda.synchronize()
        assert torch.equal(out, data) and torch.equal(out2, data) and torch.equal(par2, parity)
        assert torch.equal(batch[0], parity)
        del data, parity, par2, stripe, out, out2, batch
    torch.cuda.synchronize()
    # only descriptors and status words may stay: far below one generation of buffers (42 MiB)
    assert torch.cuda.memory_allocated() - base < 4 << 20
    assert len(rs._plans) >= 12


def test_stream_file_codec_gpu_equals_cpu_and_resumes(tmp_path):
    payload = os.urandom(5_000_011)
    g, c = tmp_path / "g", tmp_path / "c"
    g.mkdir()
    c.mkdir()
    (g / "f.bin").write_bytes(payload)
    (c / "f.bin").write_bytes(payload)
    r1 = hip().encode_file_stream(str(g / "f.bin"), 10, 4, "vandermonde", False, [0], 2, 1 << 18, 0,
                                  window=1 << 16, durable=False, stop_after=3)
    assert not r1["complete"]
    r2 = hip().encode_file_stream(str(g / "f.bin"), 10, 4, "vandermonde", False, [0], 2, 1 << 18, 0,
                                  window=1 << 17, durable=False)
    assert r2["complete"] and r2["resumed_from"] == 3 << 16
    cpu().encode_file(str(c / "f.bin"), 10, 4)
    for i in range(14):
        assert (g / f"_{i}_f.bin").read_bytes() == (c / f"_{i}_f.bin").read_bytes(), i
    assert (g / "f.bin.METADATA").read_bytes() == (c / "f.bin.METADATA").read_bytes()
    conf = g / "conf"
    ff.write_conf(str(conf), [ff.chunk_path(str(g / "f.bin"), r) for r in (4, 5, 6, 7, 8, 9, 10, 11, 12, 13)])
    r = hip().decode_file_stream(str(g / "f.bin"), str(conf), str(g / "out"), [0], 2, 1 << 18, 0,
                                 window=1 << 16, durable=False)
    assert r["complete"] and r["erased"] == 4
    assert (g / "out").read_bytes() == payload


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_gemm_host_multi_shards_on_one_gpu(devices):
    """The one-process multi-device path (one host thread per shard entry, src/encode.cu:368-429):
    repeated entries of device 0 exercise the shard split, 4 KiB alignment, remainder on the last
    shard and the thread join on a 1-GPU box."""
    k, p = 10, 4
    D = len(devices)
    C = 3 * 4096 * D + 12345  # odd, not a multiple of the shard alignment: remainder on the last entry
    rng = np.random.default_rng(D)
    host = torch.from_numpy(rng.integers(0, 256, size=(k, C), dtype=np.uint8)).pin_memory()
    par = torch.zeros((p, C), dtype=torch.uint8).pin_memory()
    e = GF256.vandermonde_ref(k, p)
    res = hip().gemm_host(devices, [host[j].data_ptr() for j in range(k)], [par[i].data_ptr() for i in range(p)],
                          e.tobytes(), C, 1, 1 << 14, 0, False)
    assert len(res["devices"]) == D
    shards = [hip().device_shard(C, D, d) for d in range(D)]
    assert shards[0][0] == 0 and shards[-1][1] == C
    assert all(a % 4096 == 0 for a, _ in shards) and all(shards[d][1] == shards[d + 1][0] for d in range(D - 1))
    for d, (a, b) in enumerate(shards):
        assert res["devices"][d]["bytes_h2d"] == k * (b - a)
        assert res["devices"][d]["lanes"] >= 1
    assert np.array_equal(par.numpy(), GF256.gemm(e, host.numpy()))


def test_prepare_pipeline_then_gemm_single_stream_double_buffers():
    """prepare_pipeline builds the workspace ahead of time; -s 1 splits the range into >= 2 slices
    so the lane's two slots alternate (H2D of slice t+1 under the kernel + D2H of slice t)."""
    k, p, C = 8, 3, 2_000_001
    h = hip()
    h.prepare_pipeline([0], k, p, C, 1, 1 << 26)
    rng = np.random.default_rng(5)
    host = torch.from_numpy(rng.integers(0, 256, size=(k, C), dtype=np.uint8)).pin_memory()
    par = torch.zeros((p, C), dtype=torch.uint8).pin_memory()
    e = rng.integers(0, 256, size=(p, k), dtype=np.uint8)
    res = h.gemm_host([0], [host[j].data_ptr() for j in range(k)], [par[i].data_ptr() for i in range(p)],
                      e.tobytes(), C, 1, 1 << 26, 0, False)
    st = res["devices"][0]
    assert st["lanes"] == 1 and st["slices"] >= 2
    assert np.array_equal(par.numpy(), GF256.gemm(e, host.numpy()))


@pytest.mark.parametrize("devices", ["0,0", "0,0,0"])
def test_rs_cli_device_list_shards(tmp_path, devices):
    """bin/RS --devices with several shard entries: per-shard "DeviceN" lines, output bit-exact with
    the CPU codec, decode through the same sharded path."""
    exe = str(binary("RS"))
    payload = os.urandom(5_000_017)
    (tmp_path / "f.bin").write_bytes(payload)
    r = subprocess.run([exe, "-k", "10", "-n", "14", "-e", "f.bin", "-s", "2", "--devices", devices], cwd=tmp_path,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    D = len(devices.split(","))
    assert all(f"Device{d}: Total GPU encoding time" in r.stdout for d in range(D)), r.stdout
    c = tmp_path / "c"
    c.mkdir()
    (c / "f.bin").write_bytes(payload)
    cpu().encode_file(str(c / "f.bin"), 10, 4)
    for i in range(14):
        assert (tmp_path / f"_{i}_f.bin").read_bytes() == (c / f"_{i}_f.bin").read_bytes(), i
    conf = tmp_path / "conf"
    ff.write_conf(str(conf), [f"_{i}_f.bin" for i in (1, 2, 4, 5, 6, 8, 10, 11, 12, 13)])
    r = subprocess.run([exe, "-d", "-i", "f.bin", "-c", "conf", "-o", "out.bin", "--devices", devices], cwd=tmp_path,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "out.bin").read_bytes() == payload


@pytest.mark.parametrize("k,n,e,C", [(10, 14, 3, 1_000_003), (4, 6, 2, 65537), (128, 160, 26, 1 << 20)])
def test_pattern_decoder_device_built_plans(k, n, e, C):
    """One PatternDecoder serves every pattern with e erased natives: the survivor list is written
    into device memory only, the kernel derives the erased natives, the row pointers and the tables
    (no host involvement), and the fused pass rebuilds + copies every native. k=128 runs the FP4
    matrix-core decode from descriptor row pointers."""
    from gpu_rscode_amd.ops import PatternDecoder

    rs = ReedSolomon(k, n)
    host, data = _data(k, C, 5)
    parity = rs.encode(data)
    out = alloc_rows(k, C, "cuda", fill=0)
    g = torch.from_numpy(rs.G).cuda()
    dec = PatternDecoder(g, [data[i] for i in range(k)] + [parity[i] for i in range(n - k)], [out[i] for i in range(k)], e)
    assert dec.engine == ("mfma" if k >= 64 else "valu")
    rng = np.random.default_rng(9)
    tested = 0
    while tested < 4:
        nat = rng.choice(k, size=e, replace=False).tolist()
        extra = rng.choice(n - k, size=min(n - k - e, 1) if n - k > e else 0, replace=False).tolist()
        erased = set(nat) | {k + x for x in extra}
        rows = [r for r in range(n) if r not in erased][:k]
        if not rs.is_recoverable(rows):
            continue
        out.zero_()
        dec.rows.copy_(torch.tensor(rows, dtype=torch.int32))
        dec.solve()
        dec.run()
        torch.cuda.synchronize()
        assert int(dec.status.item()) == 0, rows
        assert sorted(dec.erased.cpu().tolist()) == sorted(nat)
        assert np.array_equal(out.cpu().numpy(), host), rows
        tested += 1


def test_pattern_decoder_rejects_bad_patterns_without_writing():
    """Invalid survivor lists (duplicate id, id out of range, wrong number of erased natives) report
    status 2; a non-MDS singular pattern reports 1. Neither writes any output row."""
    from gpu_rscode_amd.ops import PatternDecoder

    k, n, C = 10, 14, 4099
    rs = ReedSolomon(k, n)
    host, data = _data(k, C, 6)
    parity = rs.encode(data)
    out = alloc_rows(k, C, "cuda", fill=0x5A)
    g = torch.from_numpy(rs.G).cuda()
    dec = PatternDecoder(g, [data[i] for i in range(k)] + [parity[i] for i in range(n - k)], [out[i] for i in range(k)], 4)
    # {4,5,9,11} is one of the reference Vandermonde's 12 singular 4-erasure sets: it
    # erases natives 4, 5, 9 and parity 11, so it runs on a 3-native plan
    singular = [r for r in range(n) if r not in (4, 5, 9, 11)]
    assert not rs.is_recoverable(singular)
    cases = {2: [[0, 0, 2, 3, 6, 7, 8, 10, 11, 12],  # duplicate id
                 [0, 1, 2, 3, 6, 7, 8, 10, 11, 99],  # id out of range
                 [0, 1, 2, 3, 4, 6, 7, 8, 10, 11]],  # 2 natives missing, the plan rebuilds 4
             1: [singular]}
    dec3 = PatternDecoder(g, [data[i] for i in range(k)] + [parity[i] for i in range(n - k)], [out[i] for i in range(k)], 3)
    for want, pats in cases.items():
        for rows in pats:
            d = dec3 if want == 1 else dec
            d.rows.copy_(torch.tensor(rows, dtype=torch.int32))
            d.solve()
            d.run()
            torch.cuda.synchronize()
            assert int(d.status.item()) == want, rows
            assert bool((out == 0x5A).all()), rows  # nothing stored: no output or copy pointer


def test_distributed_rs_on_a_one_rank_rccl_group():
    """DistributedRS with a forced one-rank RCCL ("nccl") group on the MI355X: broadcast_matrix, the
    scatter (odd C: rank 0's shard is re-pitched through send/recv to itself) and the in-place gather
    all execute as RCCL calls."""
    code = r'''
import os, numpy as np, torch, torch.distributed as dist
from gpu_rscode_amd.parallel import dist as pdist
from gpu_rscode_amd.gf import GF256
ctx = pdist.init_distributed(force_pg=True)
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
k, n, C = 10, 14, 5 * 4096 + 77
drs = pdist.DistributedRS(k, n, ctx)
host = np.random.default_rng(0).integers(0, 256, size=(k, C), dtype=np.uint8)
data = torch.from_numpy(host).cuda()
parity = drs.encode_global(data, C)
torch.cuda.synchronize()
assert np.array_equal(parity.cpu().numpy(), GF256.gemm(GF256.vandermonde_ref(k, n - k), host))
stripe = torch.cat([data, parity.contiguous()])
rows = [0, 1, 3, 5, 6, 8, 10, 11, 12, 13]
out = drs.decode_global(stripe[rows].contiguous(), rows, C)
torch.cuda.synchronize()
assert np.array_equal(out.cpu().numpy(), host)
dist.destroy_process_group()
print("DRS-RCCL-OK")
'''
    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=180, env=env, cwd=root)
    assert r.returncode == 0 and "DRS-RCCL-OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


def test_distributed_rs_gf65536_on_a_one_rank_rccl_group():
    """DistributedRS(field="gf65536") on a forced one-rank RCCL group: E and the survivor ids (here
    up to 269, past a byte) travel as int32 RCCL broadcasts, the stripe through the RCCL scatter and
    gather, the codec on the GPU's GF(2^16) kernels; bit-exact against the single-process codec."""
    code = r'''
import numpy as np, torch, torch.distributed as dist
from gpu_rscode_amd.parallel import dist as pdist
from gpu_rscode_amd.models import ReedSolomon
ctx = pdist.init_distributed(force_pg=True)
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
k, n, C = 250, 270, 3 * 4096 + 78
drs = pdist.DistributedRS(k, n, ctx, field="gf65536")
ref = ReedSolomon(k, n, field="gf65536")
host = np.random.default_rng(5).integers(0, 256, size=(k, C), dtype=np.uint8)
data = torch.from_numpy(host).cuda()
parity = drs.encode_global(data, C)
torch.cuda.synchronize()
want = torch.zeros((n - k, C), dtype=torch.uint8)
ref.encode(torch.from_numpy(host), want)
assert torch.equal(parity.cpu(), want)
stripe = torch.cat([data, parity.contiguous()])
rows = list(range(20, k)) + list(range(k, n))
out = drs.decode_global(stripe[rows].contiguous(), rows, C)
torch.cuda.synchronize()
assert np.array_equal(out.cpu().numpy(), host)
dist.destroy_process_group()
print("DRS16-RCCL-OK")
'''
    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=180, env=env, cwd=root)
    assert r.returncode == 0 and "DRS16-RCCL-OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


def test_host_pipeline_rows_beyond_the_2d_pitch_cap_copy_row_by_row():
    """Equally spaced host rows whose pitch exceeds the 2-D copy cap (2^31 - 1; lowered here with
    GFRS_TUNE=max_rect_pitch) move as per-row copies and still encode exactly."""
    code = r'''
import numpy as np, torch
from gpu_rscode_amd._native import hip
from gpu_rscode_amd.gf import GF256
k, p, C = 10, 4, 300_007
host = torch.from_numpy(np.random.default_rng(3).integers(0, 256, size=(k, C), dtype=np.uint8)).pin_memory()
par = torch.zeros((p, C), dtype=torch.uint8).pin_memory()
e = GF256.vandermonde_ref(k, p)
hip().gemm_host([0], [host[j].data_ptr() for j in range(k)], [par[i].data_ptr() for i in range(p)], e.tobytes(), C, 2,
                1 << 16, 0, False)
assert np.array_equal(par.numpy(), GF256.gemm(e, host.numpy()))
print("PITCH-CAP-OK")
'''
    env = dict(os.environ, GFRS_TUNE="max_rect_pitch=4096")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=180, env=env, cwd=root)
    assert r.returncode == 0 and "PITCH-CAP-OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


def test_host_pipeline_gf16_nibble_method():
    """gemm_host(field_w=4): the GF(16) method (doc/design.tex:190-209) through the pinned streaming
    pipeline, checked against the numpy GF(16) nibble maps."""
    k, p, C = 4, 2, 1_000_003
    rs = ReedSolomon(k, k + p, field="gf16")
    host = torch.from_numpy(np.random.default_rng(16).integers(0, 256, size=(k, C), dtype=np.uint8)).pin_memory()
    par = torch.zeros((p, C), dtype=torch.uint8).pin_memory()
    hip().gemm_host([0], [host[j].data_ptr() for j in range(k)], [par[i].data_ptr() for i in range(p)],
                    np.ascontiguousarray(rs.E).tobytes(), C, 2, 1 << 18, 0, False, field_w=4)
    maps = rs._maps(rs.E)
    want = np.zeros((p, C), np.uint8)
    for i in range(p):
        for j in range(k):
            want[i] ^= maps[i, j][host[j].numpy()]
    assert np.array_equal(par.numpy(), want)


def _pitched_pinned(rows, C, pitch=4096):
    P = (C + pitch - 1) // pitch * pitch
    base = torch.zeros(rows * P, dtype=torch.uint8).pin_memory()
    return base.as_strided((rows, C), (P, 1))


@pytest.mark.parametrize("field_w", [8, 16])
def test_zero_copy_pipeline_matches_staged_and_oracle(field_w):
    """zero_copy: the GEMM kernel reads the pinned host rows and writes the parity rows over PCIe
    itself (no slice buffers, no copy engines). 4 KiB-pitched rows take it; a contiguous odd-C
    buffer (unaligned rows) falls back to the staged pipeline, with the same bytes."""
    from gpu_rscode_amd import gf
    from gpu_rscode_amd.ops.gemm import _pack16

    k, p = 10, 4
    C = 3_000_018 if field_w == 16 else 3_000_017
    rng = np.random.default_rng(field_w)
    host = _pitched_pinned(k, C)
    host.copy_(torch.from_numpy(rng.integers(0, 256, size=(k, C), dtype=np.uint8)))
    h = hip()
    if field_w == 16:
        e = rng.integers(0, 65536, size=(p, k))
        coeff = _pack16(e)
        want = gf.field(16).gemm(e, host.numpy().copy().view("<u2")).view(np.uint8)
    else:
        e = GF256.vandermonde_ref(k, p)
        coeff = e.tobytes()
        want = GF256.gemm(e, host.numpy())
    outs = {}
    for zc in (True, False):
        par = _pitched_pinned(p, C)
        res = h.gemm_host([0], [host[j].data_ptr() for j in range(k)], [par[i].data_ptr() for i in range(p)],
                          coeff, C, 2, 1 << 20, 0, False, field_w=field_w, zero_copy=zc)
        assert res["devices"][0]["zero_copy"] is zc
        outs[zc] = par.numpy().copy()
    assert np.array_equal(outs[True], want) and np.array_equal(outs[False], want)
    if field_w == 8:  # unaligned rows: staged fallback
        flat = torch.from_numpy(rng.integers(0, 256, size=(k, C), dtype=np.uint8)).pin_memory()
        par = torch.zeros((p, C), dtype=torch.uint8).pin_memory()
        res = h.gemm_host([0], [flat[j].data_ptr() for j in range(k)], [par[i].data_ptr() for i in range(p)],
                          coeff, C, 2, 1 << 20, 0, False, zero_copy=True)
        assert res["devices"][0]["zero_copy"] is False
        assert np.array_equal(par.numpy(), GF256.gemm(e, flat.numpy()))


def test_rs_cli_zero_copy_roundtrip(tmp_path):
    exe = str(binary("RS"))
    payload = os.urandom(10_000_019)
    (tmp_path / "f.bin").write_bytes(payload)
    r = subprocess.run([exe, "-k", "10", "-n", "14", "-e", "f.bin", "--zero-copy"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "zero-copy kernel" in r.stdout
    g = tmp_path / "g"
    g.mkdir()
    (g / "f.bin").write_bytes(payload)
    cpu().encode_file(str(g / "f.bin"), 10, 4)
    for i in range(14):
        assert (tmp_path / f"_{i}_f.bin").read_bytes() == (g / f"_{i}_f.bin").read_bytes(), i
    ff.write_conf(str(tmp_path / "conf"), ff.worst_case_conf("f.bin", 14, 10))
    r = subprocess.run([exe, "-d", "-i", "f.bin", "-c", "conf", "-o", "o.bin", "--zero-copy"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "o.bin").read_bytes() == payload


def test_zero_copy_path_is_reported_per_device():
    """gemm_host over devices [0, 0] (two shards, one thread each): with every row pinned both shards
    run the zero-copy kernel; with one pageable (unregistered) input row each device reports the
    staged pipeline and why; a wide code (more outputs than one tile) is refused the same way. The
    bytes stay bit-exact on every path."""
    k, p, C = 8, 3, 2 * 4096 * 33 + 4096
    rng = np.random.default_rng(11)
    host = _pitched_pinned(k, C)
    host.copy_(torch.from_numpy(rng.integers(0, 256, size=(k, C), dtype=np.uint8)))
    e = GF256.vandermonde_ref(k, p)
    h = hip()

    def run(rows, m, coeff):
        par = _pitched_pinned(m, C)
        res = h.gemm_host([0, 0], [r.data_ptr() for r in rows], [par[i].data_ptr() for i in range(m)],
                          coeff.tobytes(), C, 2, 1 << 20, 0, False, zero_copy=True)
        return res["devices"], par.numpy().copy()

    devs, par = run([host[j] for j in range(k)], p, e)
    assert [d["zero_copy"] for d in devs] == [True, True] and all(d["zero_copy_refused"] == "" for d in devs)
    assert np.array_equal(par, GF256.gemm(e, host.numpy()))
    pageable = torch.empty(C + 64, dtype=torch.uint8)  # not registered with HIP: not device-mapped
    off = (-pageable.data_ptr()) % 16
    row3 = pageable[off:off + C]
    row3.copy_(host[3])
    devs, par = run([host[j] if j != 3 else row3 for j in range(k)], p, e)
    assert [d["zero_copy"] for d in devs] == [False, False]
    assert all("not mapped" in d["zero_copy_refused"] for d in devs)
    assert np.array_equal(par, GF256.gemm(e, host.numpy()))
    wide = rng.integers(0, 256, size=(20, k)).astype(np.uint8)  # m_pad 32 > one 16-row tile
    devs, par = run([host[j] for j in range(k)], 20, wide)
    assert [d["zero_copy"] for d in devs] == [False, False] and all("tile" in d["zero_copy_refused"] for d in devs)
    assert np.array_equal(par, GF256.gemm(wide, host.numpy()))


@pytest.mark.parametrize("C,B", [(8_192, 5), (3 * 256 + 77, 3), (1_000, 2)])
def test_batched_wide_code_on_matrix_cores(C, B):
    """RS(128,160) objects in one [B, k, C] allocation take the batched FP4 launch (one persistent
    grid over every stripe's chunks, the A-resident kernel), ragged remainders on the batched v_perm
    kernel: encode_batch and decode_batch (26 natives + 6 parity lost, survivors copied in the same
    pass) bit-exact against the oracle on every stripe; scattered stripes stay on the v_perm path."""
    from gpu_rscode_amd.ops import GemmPlan

    k, n = 128, 160
    rs = ReedSolomon(k, n, matrix="cauchy")
    host = np.random.default_rng(C + B).integers(0, 256, size=(B, k, C), dtype=np.uint8)
    P = (C + 255) // 256 * 256  # 16-byte aligned rows (a ragged C pitched up), one allocation

    def pitched(rows):
        return torch.empty((B, rows, P), dtype=torch.uint8, device="cuda")[:, :, :C]
    data = pitched(k)
    data.copy_(torch.from_numpy(host))
    parity = rs.encode_batch(data)
    torch.cuda.synchronize()
    plan = [p for key, p in rs._plans.items() if key[0] == "encb"][0]
    assert plan.engine == "mfma" and plan.in_bstride == k * P
    for b in range(B):
        assert np.array_equal(parity[b].cpu().numpy(), GF256.gemm(rs.E, host[b])), b
    lost = set(range(0, 128, 5)) | {128, 133, 140, 149, 155, 159}
    rows = [r for r in range(n) if r not in lost][:k]
    stripe = torch.cat([data, parity], dim=1)
    surv = pitched(k)
    surv.copy_(stripe[:, rows])
    out = rs.decode_batch(surv, rows, pitched(k))
    torch.cuda.synchronize()
    dplan = [p for key, p in rs._plans.items() if key[0] == "decb"][0]
    assert dplan.engine == "mfma" and dplan.has_copies
    assert torch.equal(out, data)
    # stripes in separate allocations, not equally spaced: the v_perm batched kernel
    ins = [alloc_rows(k, C, "cuda") for _ in range(2)]
    pad = torch.empty(12345, dtype=torch.uint8, device="cuda")  # noqa: F841 (breaks the spacing)
    ins.append(alloc_rows(k, C, "cuda"))
    for i in ins:
        i.copy_(torch.from_numpy(host[0]))
    outs = [alloc_rows(n - k, C, "cuda") for _ in ins]
    ptrs = [int(x.data_ptr()) for x in ins]
    p2 = GemmPlan([[r for r in x] for x in ins], [[r for r in o] for o in outs], rs.E)
    if ptrs[1] - ptrs[0] != ptrs[2] - ptrs[1]:
        assert p2.engine == "valu"
    p2.run()
    torch.cuda.synchronize()
    assert all(np.array_equal(o.cpu().numpy(), GF256.gemm(rs.E, host[0])) for o in outs)
