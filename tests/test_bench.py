"""bench.py driver contract on the host: the --gpus launcher (re-launch through torch.distributed.run
as a child), the WORLD_SIZE check, the per-step parity exchange of every --comm mode over gloo, and
the one-line JSON record. The same code runs over RCCL on MI355X (--device cuda, the default)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=300):
    e = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(v, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=e, cwd=ROOT)


def _record(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out  # exactly one JSON line, from rank 0
    return json.loads(lines[0])


@pytest.mark.parametrize("gpus", [2, 3])
def test_launcher_runs_world_ranks_and_reports_every_comm_mode(gpus):
    r = _run(["--device", "cpu", "--gpus", str(gpus), "--steps", "3", "--warmup", "1", "--bytes", str(300_001)])
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _record(r.stdout)
    assert rec["n_gpus"] == gpus and rec["steps"] == 3 and rec["warmup"] == 1
    assert rec["verified"] is True
    assert rec["config"]["comm"] == "owners" and rec["config"]["parallelism"].startswith(f"dp{gpus}")
    by = rec["value_by_comm"]
    assert set(by) == {"owners", "root", "none"} and all(v["verified"] for v in by.values())
    par_bytes = by["owners"]["bytes_sent_per_rank_step"]
    assert par_bytes > 0 and by["none"]["bytes_sent_per_rank_step"] == 0
    assert by["root"]["bytes_recv_rank0_step"] > par_bytes  # rank 0 takes whole blocks from every peer
    assert rec["value"] == by["owners"]["GBps"] and rec["value_no_comm"] == by["none"]["GBps"]
    # busiest link: one piece per ordered pair (owners) vs a whole block into rank 0 (root)
    assert by["root"]["busiest_link_bytes_per_step"] > by["owners"]["busiest_link_bytes_per_step"] > 0
    assert by["none"]["busiest_link_bytes_per_step"] == 0 and by["owners"]["busiest_link_GBps_implied"] > 0


def test_single_rank_record_and_comm_choice():
    r = _run(["--device", "cpu", "--steps", "2", "--warmup", "1", "--comm", "root"])
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _record(r.stdout)
    assert rec["n_gpus"] == 1 and rec["config"]["comm"] == "none" and "value_by_comm" not in rec
    for key in ("metric", "value", "unit", "ms_per_step", "higher_is_better", "scaling", "vs_baseline", "dtype", "data"):
        assert key in rec


def test_world_size_mismatch_is_an_error():
    r = _run(["--device", "cpu", "--gpus", "3", "--steps", "1"], env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("preset,erased", [("k10n14", 4), ("k128n160", 32)])
def test_gpu_bench_record_with_worst_case_e2e_decode(preset, erased):
    """One rank on the MI355X, 64 MiB: the device step verifies, and the e2e block's decode rebuilds
    the first `erasures` natives (src/unit-test.sh keeps the last k chunks) through the host pipeline."""
    r = _run(["--preset", preset, "--steps", "3", "--warmup", "1", "--bytes", str(64 << 20)], timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _record(r.stdout)
    assert rec["verified"] is True and rec["n_gpus"] == 1 and rec["config"]["device"] == "cuda"
    assert rec["config"]["engine"] == ("mfma" if preset == "k128n160" else "valu")
    e2e = rec["e2e"]
    assert e2e["verified"] is True and e2e["erased"] == erased
    assert e2e["encode_GBps"] > 0 and e2e["decode_GBps"] > 0
