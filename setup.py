"""pip packaging (reference python/framework/setup.py builds libpccl with CMake as part of the wheel).

    pip install .            # builds libpccl.so / libpccl_hip.so (gfx950) / ccoip_master with CMake + Ninja
    PCCL_BUILD_HIP_SUPPORT=0 pip install .   # CPU-only build

Installs the ``pccl_amd`` package (plus the ``pccl`` alias) with the native libraries in ``pccl_amd/lib`` and the
``pccl_master`` console script.
"""
import os
import subprocess

from setuptools import setup
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))


class CMakeBuild(build_py):
    def run(self):
        bdir = os.path.join(ROOT, "build")
        hip = os.environ.get("PCCL_BUILD_HIP_SUPPORT", "1")
        subprocess.check_call(["cmake", "-S", ROOT, "-B", bdir, "-G", "Ninja", "-DCMAKE_BUILD_TYPE=Release",
                               f"-DPCCL_BUILD_HIP_SUPPORT={'ON' if hip == '1' else 'OFF'}", "-DPCCL_BUILD_TESTS=OFF"])
        subprocess.check_call(["ninja", "-C", bdir])
        super().run()


setup(
    name="pccl-amd",
    version="0.1.0",
    description="MI355X-native fault-tolerant collective communications (PCCL-compatible API)",
    packages=["pccl_amd", "pccl_amd.ops", "pccl_amd.parallel", "pccl_amd.models", "pccl_amd.utils", "pccl"],
    package_data={"pccl_amd": ["lib/*.so", "lib/ccoip_master"]},
    include_package_data=True,
    python_requires=">=3.9",
    install_requires=["numpy"],
    extras_require={"torch": ["torch"]},
    entry_points={"console_scripts": ["pccl_master=pccl_amd.master:main"]},
    cmdclass={"build_py": CMakeBuild},
)
