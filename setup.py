"""setuptools hook: build the native extensions in-tree (hipcc for gfx950 + g++) before
the package files are collected, so wheels and editable installs carry _hip_ops.so and
_lsnative.so.  ``LANGSTREAM_GPU_ARCH`` selects the offload arch (default gfx950)."""
from setuptools import setup
from setuptools.command.build_py import build_py


class BuildNative(build_py):
    def run(self):
        import os
        import sys
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from langstream_amd import _build
        _build.build_all(verbose=True)
        super().run()


setup(cmdclass={"build_py": BuildNative})
