"""pip entry: builds dgraph_amd/_C.so for gfx950 (``dgraph_amd._build``) before packaging.

``pip install -e .`` / ``pip wheel .`` run the same in-tree hipcc build as
``python -m dgraph_amd._build``; set ``DGRAPH_SKIP_NATIVE_BUILD=1`` to package an
already-built library (or none: CPU-only use of the pure-PyTorch reference ops).
"""
import os

from setuptools import setup
from setuptools.command.build_py import build_py


class BuildWithNative(build_py):
    def run(self):
        if not os.environ.get("DGRAPH_SKIP_NATIVE_BUILD"):
            from dgraph_amd import _build

            _build.build(verbose=True)
        super().run()


setup(cmdclass={"build_py": BuildWithNative})
