"""Lint the emitted gfx950 code of the FP4 matrix-core kernels (no GPU needed: hipcc cross-compiles).

The epilogues read MFMA accumulators through an inline-asm ``v_bfi_b32`` that the compiler's hazard
recognizer does not see into; a read too soon after the last MFMA returned stale accumulator bits on
the MI355X (gf_mfma16.hip with one M-tile per block). ``scripts/mfma_hazard_check.py`` walks the
assembly and counts the issue slots between each such read and the MFMA that wrote its registers.
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("name", ["gf_mfma16", "gf_mfma_fp4", "gf_mfma_fp4ar", "gf_mfma_fp4tm"])
def test_no_unguarded_accumulator_reads(name, tmp_path):
    asm = tmp_path / f"{name}.s"
    # (compiled as csrc/Makefile does: the A-resident and tile-major kernels in MFMA VGPR form)
    extra = ["-mllvm", "-amdgpu-mfma-vgpr-form=1"] if name in ("gf_mfma_fp4ar", "gf_mfma_fp4tm") else []
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-S", "--offload-device-only", *extra,
                    "-I", os.path.join(ROOT, "csrc", "include"), os.path.join(ROOT, "csrc", "kernels", f"{name}.hip"),
                    "-o", str(asm)], check=True, capture_output=True, timeout=600)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "mfma_hazard_check.py"), str(asm)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:]
