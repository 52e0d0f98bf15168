"""The native-module loader: make runs only for a stale module, under a cross-process lock.

torchrun starts every rank at once; a snapshot without make's intermediate objects (build/) used to
make each rank relink _cpu.so while its peers imported it ("dynamic module does not define module
export function"). The loader now imports an up-to-date module as it is.
"""
import multiprocessing as mp
import time

from gpu_rscode_amd import _build, _native


def _fresh(monkeypatch, stale):
    calls = []
    monkeypatch.setattr(_native, "_mods", {})
    monkeypatch.delenv("GPURS_NO_BUILD", raising=False)
    monkeypatch.setattr(_build, "stale", lambda p: stale)
    monkeypatch.setattr(_build, "build", lambda target: calls.append(target))
    return calls


def test_up_to_date_module_is_imported_without_make(monkeypatch):
    calls = _fresh(monkeypatch, stale=False)
    assert hasattr(_native.cpu(), "encoding_matrix")
    assert calls == []


def test_stale_module_is_rebuilt_once(monkeypatch):
    calls = _fresh(monkeypatch, stale=True)
    try:
        _native.cpu()
    except Exception:
        pass  # the patched staleness never clears; only the build call matters here
    assert calls == ["cpu"]


def _hold(q, secs):
    with _build.file_lock():
        q.put(("in", time.monotonic()))
        time.sleep(secs)
        q.put(("out", time.monotonic()))


def test_file_lock_serialises_processes():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_hold, args=(q, 0.3)) for _ in range(3)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    ev = sorted((q.get(timeout=5) for _ in range(6)), key=lambda x: x[1])
    assert [e[0] for e in ev] == ["in", "out"] * 3  # no two holders at once


def test_fp4_router_table():
    """The FP4 engine's one routing function (fp4_route, csrc/kernels/gf_mfma_fp4.hip) and its
    override (GFRS_TUNE=fp4=..., parsed among other keys): k = 128 wide-stripe shapes by M-tile count, plain and with fused copies."""
    import os

    from gpu_rscode_amd._native import hip

    h = hip()
    want = {(8, False): "v1", (12, True): "v1", (16, False): "ar", (16, True): "ar", (20, False): "tm",
            (20, True): "tm", (24, False): "tm", (24, True): "tm", (28, True): "tm", (28, False): "tm",
            (32, False): "ar", (32, True): "tm", (40, False): "v1"}
    for (m, copy), form in want.items():
        assert h.fp4_route(128, m, copy, 8) == form, (m, copy)
    assert h.fp4_route(100, 17, False, 8) == "v1"  # k outside (112, 128]
    os.environ["GFRS_TUNE"] = "fp4=v1"
    try:
        assert h.fp4_route(128, 28, True, 8) == "tm"  # (no v1 build for 7 tiles: the routed form)
        assert h.fp4_route(128, 16, True, 8) == "v1"
        assert h.fp4_route(128, 24, True, 8) == "v1"
        assert h.fp4_route(128, 32, True, 8) == "v1"
        os.environ["GFRS_TUNE"] = "tm8=0"
        assert h.fp4_route(128, 32, True, 8) == "v1"
        assert h.fp4_route(128, 32, False, 8) == "ar"
        os.environ["GFRS_TUNE"] = "ksplit_lanes=5,fp4=tm"
        assert h.fp4_route(128, 24, True, 8) == "tm"
        assert h.fp4_route(128, 12, True, 8) == "v1"  # (not built for 3 tiles: the routed form)
        assert h.fp4_route(128, 16, False, 8) == "ar"  # (not built for 4 tiles: the routed form)
    finally:
        del os.environ["GFRS_TUNE"]
