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
    assert rec["verified"] is True and rec["scaling"] == "weak" and "headline_why" in rec
    assert rec["config"]["comm"] == "bcast" and rec["config"]["parallelism"].startswith(f"dp{gpus}")
    by = rec["value_by_comm"]
    assert set(by) == {"bcast", "owners", "root", "none"} and all(v["verified"] for v in by.values())
    par_bytes = by["owners"]["bytes_sent_per_rank_step"]
    assert par_bytes > 0 and by["none"]["bytes_sent_per_rank_step"] == 0
    assert by["bcast"]["bytes_sent_per_rank_step"] == 0  # the headline keeps parity in place
    assert by["root"]["bytes_recv_rank0_step"] > par_bytes  # rank 0 takes whole blocks from every peer
    assert rec["value"] == by["bcast"]["GBps"] and rec["value_no_comm"] == by["none"]["GBps"]
    # busiest link: one piece per ordered pair (owners) vs a whole block into rank 0 (root)
    assert by["root"]["busiest_link_bytes_per_step"] > by["owners"]["busiest_link_bytes_per_step"] > 0
    assert by["none"]["busiest_link_bytes_per_step"] == 0 and by["owners"]["busiest_link_GBps_implied"] > 0
    # the reference's strong scaling: one stripe sharded over the ranks, gathered into rank 0 per step
    st = rec["strong"]
    assert st["verified"] is True and rec["value_strong"] == st["GBps"] and len(st["shard_cols"]) == gpus
    assert sum(st["shard_cols"]) == (300_001 + 9) // 10 and st["gather"] == "step"
    assert st["bytes_recv_rank0"] == 14 * (sum(st["shard_cols"]) - st["shard_cols"][0])
    # per-rank step times of the headline loop (a straggler shows as the max)
    sm = rec["step_ms_by_rank"]
    assert len(sm["per_rank"]) == gpus and sm["max"] == max(sm["per_rank"]) and sm["max"] == rec["ms_per_step"]
    assert all(len(v["step_ms_by_rank"]) == gpus for v in by.values()) and rec["comparisons_complete"] is True


def _fault_run(mode, env, gpus=3):
    e = {"GFRS_FAULT_MODE": mode, "GFRS_COMPARE_BUDGET_S": "25", **env}
    r = _run(["--device", "cpu", "--gpus", str(gpus), "--steps", "3", "--warmup", "1", "--bytes", str(200_003)],
             env=e, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    rec = _record(r.stdout)
    assert rec["verified"] is True and rec["value"] > 0 and rec["comparisons_complete"] is False
    assert rec["value_by_comm"]["bcast"]["verified"] is True  # the headline survives
    return rec


def test_fault_in_root_mode_on_every_rank_keeps_the_headline():
    """An exception in the root gather (the last comparison) on every rank: the headline and every
    earlier mode are in the one record, root carries the error."""
    rec = _fault_run("root", {})
    by = rec["value_by_comm"]
    assert "InjectedFault" in by["root"]["error"]
    assert by["none"]["verified"] and by["owners"]["verified"] and rec["strong"]["verified"]


def test_fault_on_one_rank_stops_later_modes():
    """Rank 1 alone fails in the owners all_to_all: its peers see the collective break, owners is an
    error, the modes after it are skipped (no collective is issued on a group that may be out of
    step) and rank 0 still prints the verified headline."""
    rec = _fault_run("owners", {"GFRS_FAULT_RANK": "1"})
    by = rec["value_by_comm"]
    assert "error" in by["owners"] and by["none"]["verified"] is True
    assert "skipped" in rec["strong"] and "skipped" in by["root"]


def test_hung_peer_is_cut_off_by_the_watchdog():
    """Rank 2 never joins the strong-scaling gather (it sleeps): no collective raises, the comparison
    watchdog expires, rank 0 prints the headline with strong marked as timed out, all ranks exit 0."""
    rec = _fault_run("strong", {"GFRS_FAULT_RANK": "2", "GFRS_FAULT_KIND": "hang", "GFRS_COMPARE_BUDGET_S": "15"})
    assert "timed out" in rec["strong"]["error"] and "skipped" in rec["value_by_comm"]["root"]
    assert rec["value_by_comm"]["owners"]["verified"] is True


@pytest.mark.parametrize("gather", ["step", "end"])
def test_strong_scaling_headline(gather):
    r = _run(["--device", "cpu", "--gpus", "2", "--scaling", "strong", "--gather", gather, "--steps", "2",
              "--warmup", "1", "--bytes", str(200_003)])
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _record(r.stdout)
    assert rec["scaling"] == "strong" and rec["verified"] is True and rec["value"] == rec["value_strong"]
    assert rec["config"]["comm"] == f"strong/{gather}" and "value_by_comm" not in rec
    if gather == "end":
        assert rec["strong"]["gather_ms"] > 0


def test_forced_one_rank_group_runs_every_mode():
    r = _run(["--device", "cpu", "--force-pg", "--steps", "2", "--warmup", "1", "--bytes", str(100_000)])
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _record(r.stdout)
    assert rec["n_gpus"] == 1 and rec["config"]["process_group"] is True and rec["verified"] is True
    assert set(rec["value_by_comm"]) == {"bcast", "owners", "root", "none"} and rec["strong"]["verified"]


def test_single_rank_record_and_comm_choice():
    r = _run(["--device", "cpu", "--steps", "2", "--warmup", "1", "--comm", "root"])
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _record(r.stdout)
    assert rec["n_gpus"] == 1 and rec["config"]["comm"] == "none" and "value_by_comm" not in rec
    for key in ("metric", "value", "unit", "ms_per_step", "higher_is_better", "scaling", "vs_baseline", "dtype", "data"):
        assert key in rec


def test_prewarm_runs_local_steps_before_the_warmup():
    """--min-warmup-ms: untimed local steps until the floor has passed, recorded; the timed loop is
    still exactly --steps steps after --warmup steps (3 ranks: the pre-warm issues no collective,
    so ranks that run different counts of it must not hang)."""
    r = _run(["--device", "cpu", "--gpus", "3", "--steps", "2", "--warmup", "1", "--bytes", str(60_000),
              "--min-warmup-ms", "30", "--no-compare"])
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _record(r.stdout)
    assert rec["verified"] is True and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["prewarm"]["steps"] > 0 and rec["prewarm"]["ms"] >= 30 and rec["prewarm"]["min_ms"] == 30
    r = _run(["--device", "cpu", "--steps", "2", "--warmup", "1"])
    assert _record(r.stdout)["prewarm"]["steps"] == 0  # off by default on the CPU


def test_every_preset_parses():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    for name, pr in bench.PRESETS.items():
        a = bench.parse(["--preset", name])
        assert (a.k, a.n, a.bytes, a.erasures) == (pr["k"], pr["n"], pr["bytes"], pr["erasures"])
        assert a.scaling == pr.get("scaling", "weak") and a.lanes == pr.get("lanes", 2)
        assert a.min_warmup_ms == float(os.environ.get("GFRS_MIN_WARMUP_MS", 250))  # cuda default
    a = bench.parse(["--preset", "k16n20_64g", "--scaling", "weak", "--lanes", "2"])
    assert a.scaling == "weak" and a.lanes == 2  # explicit flags win over the preset


def test_world_size_mismatch_is_an_error():
    r = _run(["--device", "cpu", "--gpus", "3", "--steps", "1"], env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("preset,erased", [("k10n14", 4), ("k128n160", 32)])
def test_gpu_bench_record_with_worst_case_e2e_decode(preset, erased):
    """One rank on the MI355X, 64 MiB: the device step verifies, and the e2e block's decode rebuilds
    the first `erasures` natives (src/unit-test.sh keeps the last k chunks) through the host pipeline,
    and its reference-shaped decode writes all k natives into one pinned file image."""
    r = _run(["--preset", preset, "--steps", "3", "--warmup", "1", "--bytes", str(64 << 20)], timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _record(r.stdout)
    assert rec["verified"] is True and rec["n_gpus"] == 1 and rec["config"]["device"] == "cuda"
    assert rec["config"]["engine"] == ("mfma" if preset == "k128n160" else "valu")
    e2e = rec["e2e"]
    assert e2e["verified"] is True and e2e["erased"] == erased
    assert e2e["encode_GBps"] > 0 and e2e["decode_GBps"] > 0 and e2e["decode_full_GBps"] > 0


@pytest.mark.gpu
def test_gpu_bench_forced_rccl_group_every_mode():
    """--force-pg on one MI355X: a one-rank RCCL group runs the per-step pattern broadcast, the owners
    all_to_all (to self), the root grouped send/recv (to self) and the strong-scaling gather — every
    RCCL path of the N > 1 run — and each mode verifies."""
    r = _run(["--force-pg", "--steps", "4", "--warmup", "1", "--bytes", str(64 << 20), "--no-e2e"], timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _record(r.stdout)
    assert rec["verified"] is True and rec["config"]["process_group"] is True
    assert set(rec["value_by_comm"]) == {"bcast", "owners", "root", "none"}
    assert all(v["verified"] for v in rec["value_by_comm"].values()) and rec["strong"]["verified"] is True


@pytest.mark.gpu
def test_gpu_bench_strong_gather_end_one_rank_group():
    r = _run(["--force-pg", "--scaling", "strong", "--gather", "end", "--steps", "3", "--warmup", "1",
              "--bytes", str(32 << 20)], timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _record(r.stdout)
    assert rec["verified"] is True and rec["scaling"] == "strong" and rec["strong"]["gather_ms"] >= 0


@pytest.mark.gpu
def test_gpu_bench_three_ranks_rehearsed_on_one_gpu():
    """Three ranks share the one MI355X over gloo (RCCL refuses two ranks on one GPU): ranks 1 and 2
    take every step's pattern only from rank 0's look-ahead broadcast into their ring slots, and each
    decoder's last plan must match the pattern of the step it was built for. Every N > 1 mode runs:
    owners all_to_all, root's receive lists and strong scaling's per-row gather into rank 0's full
    rows (point-to-point pieces staged through host memory under gloo)."""
    r = _run(["--gpus", "3", "--pg-backend", "gloo", "--steps", "6", "--warmup", "2", "--bytes", str(32 << 20),
              "--no-e2e"], timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _record(r.stdout)
    assert rec["verified"] is True and rec["n_gpus"] == 3 and rec["config"]["pg_backend"] == "gloo"
    assert rec["config"]["rehearsal"] and set(rec["value_by_comm"]) == {"bcast", "owners", "root", "none"}
    assert all(v["verified"] for v in rec["value_by_comm"].values()) and rec["comparisons_complete"] is True
    st = rec["strong"]
    assert st["verified"] is True and len(st["shard_cols"]) == 3 and st["bytes_recv_rank0"] > 0


@pytest.mark.gpu
def test_gpu_bench_three_ranks_strong_headline_rehearsed():
    """--scaling strong as the headline with three ranks on the one GPU: one stripe column-sharded,
    every step's parity and decoded natives gathered into rank 0's full rows."""
    r = _run(["--gpus", "3", "--pg-backend", "gloo", "--scaling", "strong", "--steps", "4", "--warmup", "1",
              "--bytes", str(48 << 20)], timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _record(r.stdout)
    assert rec["verified"] is True and rec["scaling"] == "strong" and rec["strong"]["verified"] is True
    assert len(rec["step_ms_by_rank"]["per_rank"]) == 3


@pytest.mark.gpu
def test_gpu_bench_fault_in_root_mode_keeps_headline():
    """--force-pg on the MI355X with a fault injected into the root gather: one JSON line, the RCCL
    headline verified, root recorded as an error, the modes before it verified."""
    r = _run(["--force-pg", "--steps", "4", "--warmup", "1", "--bytes", str(64 << 20), "--no-e2e"],
             env={"GFRS_FAULT_MODE": "root"}, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _record(r.stdout)
    assert rec["verified"] is True and rec["comparisons_complete"] is False
    by = rec["value_by_comm"]
    assert "InjectedFault" in by["root"]["error"] and by["owners"]["verified"] and rec["strong"]["verified"]


@pytest.mark.gpu
def test_gpu_bench_graph_replay_verifies():
    """--graph: every pattern's step captured once, replayed in the pool's order for more steps than
    the pool holds; the record must still verify each decoder against the last pattern it ran."""
    r = _run(["--graph", "--no-e2e", "--steps", "21", "--warmup", "2", "--bytes", str(64 << 20)], timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    rec = _record(r.stdout)
    assert rec["verified"] is True and rec["config"]["graph"] is True


def test_configs_children_embed_records_and_survive_a_crash_and_a_hang():
    """N = 1: each --configs preset runs in a fresh child process after the headline; the records
    are embedded under configs. A child that crashes (rc 7) or hangs (killed at its timeout) is
    recorded as an error and the headline record is unchanged and verified."""
    r = _run(["--device", "cpu", "--steps", "2", "--warmup", "1", "--configs", "k4n6,k10n14_w16",
              "--config-steps", "3", "--config-warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _record(r.stdout)
    cf = rec["configs"]
    assert set(cf) == {"k4n6", "k10n14_w16"} and rec["verified"] is True
    assert all(c["verified"] is True and c["steps"] == 3 and c["warmup"] == 1 and c["value"] > 0 for c in cf.values())
    assert "GF(2^16)" in cf["k10n14_w16"]["metric"] and cf["k10n14_w16"]["dtype"].startswith("uint16")
    r = _run(["--device", "cpu", "--steps", "2", "--warmup", "1", "--configs", "k4n6,k10n14_w16",
              "--config-steps", "2", "--configs-budget", "40"],
             env={"GFRS_CONFIG_FAULT": "k4n6:crash"})
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _record(r.stdout)
    assert rec["verified"] is True and rec["value"] > 0
    assert rec["configs"]["k4n6"]["rc"] == 7 and "error" in rec["configs"]["k4n6"]
    assert rec["configs"]["k10n14_w16"]["verified"] is True
    r = _run(["--device", "cpu", "--steps", "2", "--warmup", "1", "--configs", "k10n14_w16,k4n6",
              "--config-steps", "2", "--configs-budget", "25"],
             env={"GFRS_CONFIG_FAULT": "k10n14_w16:hang"}, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _record(r.stdout)
    assert rec["verified"] is True
    assert "timed out" in rec["configs"]["k10n14_w16"]["error"]
    assert "skipped" in rec["configs"]["k4n6"] or rec["configs"]["k4n6"].get("verified") is True


def test_configs_default_only_for_the_headline():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod2", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.parse([]).configs == list(bench.CONFIG_PRESETS)
    assert bench.parse(["--bytes", str(64 << 20)]).configs == []
    assert bench.parse(["--preset", "k128n160"]).configs == []
    assert bench.parse(["--device", "cpu"]).configs == []
    assert bench.parse(["--configs", "none"]).configs == []
    assert bench.parse(["--configs", "k4n6"]).configs == ["k4n6"]
