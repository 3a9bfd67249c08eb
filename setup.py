"""setup.py: builds the native extensions in-tree (ddl_amd/_build.py) before packaging.

``pip install -e .`` / ``python setup.py build_ext --inplace`` both compile
``_ddl_runtime`` (g++) and ``_ddl_hip`` (hipcc --offload-arch=gfx950).
"""

from setuptools import setup
from setuptools.command.build_ext import build_ext
from setuptools.command.build_py import build_py


class NativeBuild(build_ext):
    def run(self):
        from ddl_amd import _build

        _build.build_all()


class BuildPy(build_py):
    def run(self):
        self.run_command("build_ext")
        super().run()


setup(cmdclass={"build_ext": NativeBuild, "build_py": BuildPy})
