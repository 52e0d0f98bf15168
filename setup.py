"""``pip install --no-build-isolation .`` — builds the native modules and CLIs for gfx950 with
``make -C csrc`` (hipcc + g++) before packaging; The bin/RS and
bin/CPU-RS CLIs install into the environment's bin directory next to the ``gpu-rscode`` entry point,
the C API (lib/libgfrs.so, include/gfrs.h) into its lib and include directories.
No network is needed: --no-build-isolation uses the setuptools, wheel and pybind11 already installed."""
import os
import subprocess

from setuptools import setup
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))


class BuildNative(build_py):
    def run(self):
        jobs = str(min(8, os.cpu_count() or 4))
        subprocess.run(["make", "-C", os.path.join(ROOT, "csrc"), f"-j{jobs}", "all"], check=True)
        super().run()


setup(
    name="gpu-rscode-amd",
    version="0.2.0",
    description="Reed-Solomon erasure coding on AMD Instinct MI355X (gfx950): HIP kernels, native runtime, "
                "RCCL multi-GPU",
    python_requires=">=3.10",
    install_requires=["numpy", "torch"],
    packages=["gpu_rscode_amd", "gpu_rscode_amd.models", "gpu_rscode_amd.ops", "gpu_rscode_amd.parallel",
              "gpu_rscode_amd.utils"],
    package_data={"gpu_rscode_amd": ["_hip.so", "_cpu.so"]},
    entry_points={"console_scripts": ["gpu-rscode = gpu_rscode_amd.utils.cli:main"]},
    data_files=[("bin", ["bin/RS", "bin/CPU-RS"]), ("lib", ["lib/libgfrs.so"]), ("include", ["csrc/include/gfrs.h"])],
    cmdclass={"build_py": BuildNative},
)
