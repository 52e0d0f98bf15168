"""Packaging: `pip install --no-build-isolation .` (offline) builds the native modules with
`make -C csrc` and installs a package that works away from the source tree — no csrc/ next to it,
so it never tries to rebuild — plus the `gpu-rscode` entry point and the bin/RS, bin/CPU-RS CLIs
(the reference installs its RS binary with autotools `make install`)."""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _source_copy(dst):
    """The installable part of the tree, mtimes kept (copy2) so `make` finds everything up to date and
    pip's in-tree build files (build/lib, *.egg-info) land in the copy, not in the repository."""
    ignore = shutil.ignore_patterns("__pycache__", "*.egg-info")
    for d in ("csrc", "gpu_rscode_amd", "bin", "lib", os.path.join("build", "obj")):
        if os.path.isdir(os.path.join(ROOT, d)):
            shutil.copytree(os.path.join(ROOT, d), os.path.join(dst, d), ignore=ignore, copy_function=shutil.copy2)
    for f in ("setup.py", "pyproject.toml", "README.md"):
        shutil.copy2(os.path.join(ROOT, f), os.path.join(dst, f))


def test_pip_install_outside_the_tree(tmp_path):
    src, target = tmp_path / "src", tmp_path / "site"
    _source_copy(str(src))
    r = subprocess.run([sys.executable, "-m", "pip", "install", "--no-build-isolation", "--no-deps", "--no-index",
                        "--target", str(target), str(src)], capture_output=True, text=True, timeout=850)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert (target / "gpu_rscode_amd" / "_cpu.so").exists() and (target / "gpu_rscode_amd" / "_hip.so").exists()
    assert (target / "bin" / "RS").exists() and (target / "bin" / "CPU-RS").exists()
    # the C API: header into <prefix>/include, library into <prefix>/lib (pip's --target keeps only
    # the package part of lib/, so the library is checked in the wheel's RECORD)
    assert (target / "include" / "gfrs.h").exists()
    record = (target / "gpu_rscode_amd-0.2.0.dist-info" / "RECORD").read_text()
    assert "libgfrs.so," in record
    env = dict(os.environ, PYTHONPATH=str(target))
    code = ("import numpy as np, torch, gpu_rscode_amd\n"
            "from gpu_rscode_amd import ReedSolomon, gf\n"
            f"assert gpu_rscode_amd.__file__.startswith({str(target)!r})\n"
            "rs = ReedSolomon(10, 14)\n"
            "d = torch.randint(0, 256, (10, 4099), dtype=torch.uint8)\n"
            "p = rs.encode(d)\n"
            "assert np.array_equal(p.numpy(), gf.GF256.gemm(rs.E, d.numpy()))\n"
            "print('installed-ok')\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, cwd=tmp_path, timeout=300)
    assert r.returncode == 0 and "installed-ok" in r.stdout, r.stderr[-3000:]
    r = subprocess.run([str(target / "bin" / "gpu-rscode"), "-h"], capture_output=True, text=True, env=env,
                       cwd=tmp_path, timeout=120)
    assert r.returncode == 0 and "usage" in r.stdout.lower(), r.stderr[-2000:]
