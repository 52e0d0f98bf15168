"""The shipped examples run end to end: on the CPU codec here (bin/CPU-RS, CPU tensors) and on the
HIP path (bin/RS, cuda tensors) on an MI355X box. Each script checks its own round trip and exits
non-zero on a mismatch; the tests also look for the scripts' success lines."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples")
CASES = [
    (["bash", os.path.join(EX, "encode_decode.sh")], "identity decode OK"),
    (["bash", os.path.join(EX, "streaming_resume.sh")], "streamed round trip OK"),
    ([sys.executable, os.path.join(EX, "python_api.py")], "python API tour OK"),
    ([sys.executable, os.path.join(EX, "distributed.py")], "distributed tour OK"),
]


def _run(cmd, cwd, env_extra=None):
    env = dict(os.environ, **(env_extra or {}))
    return subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=300)


@pytest.mark.parametrize("cmd,expect", CASES, ids=["encode_decode", "streaming_resume", "python_api", "distributed"])
def test_example_cpu(cmd, expect, tmp_path):
    r = _run(cmd, tmp_path, {"HIP_VISIBLE_DEVICES": "", "CUDA_VISIBLE_DEVICES": ""})
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert expect in r.stdout
    if cmd[0] == "bash":
        assert "round trip OK with " in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("cmd,expect", CASES, ids=["encode_decode", "streaming_resume", "python_api", "distributed"])
def test_example_gpu(cmd, expect, tmp_path):
    r = _run(cmd, tmp_path)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert expect in r.stdout
    if cmd[0] == sys.executable:
        assert "on cuda" in r.stdout
    else:  # the shell examples pick the HIP CLI when a GPU is visible
        assert "round trip OK with " in r.stdout and "CPU-RS" not in r.stdout
