"""setuptools entry: `pip install .` compiles the gfx950 native library in-tree
(mxllm/_C.so, via mxllm._build — hipcc for csrc/kernels/*.hip, g++ for the
C++ runtime and torch bindings) before packaging it."""
import os
import sys

from setuptools import setup
from setuptools.command.build_py import build_py


class BuildWithNative(build_py):
    def run(self):
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from mxllm import _build

        _build.build(jobs=int(os.environ.get("MAX_JOBS", "8")), verbose=True)
        super().run()


setup(cmdclass={"build_py": BuildWithNative})
