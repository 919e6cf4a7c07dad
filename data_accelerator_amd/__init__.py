"""Distribution-name alias: ``import data_accelerator_amd.engine.query`` is ``dxa.engine.query``.

The implementation lives in the short package ``dxa``; every submodule is importable under both names (the same
module objects, so state such as ``dxa.parallel``'s process group is shared)."""
import importlib
import importlib.abc
import importlib.util
import sys

import dxa as _dxa

_PREFIX = __name__ + "."


class _AliasFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def find_spec(self, fullname, path=None, target=None):
        if fullname.startswith(_PREFIX):
            return importlib.util.spec_from_loader(fullname, self)
        return None

    def create_module(self, spec):
        return importlib.import_module("dxa." + spec.name[len(_PREFIX):])

    def exec_module(self, module):
        pass


sys.meta_path.insert(0, _AliasFinder())
__path__ = []                     # a package, so submodule imports reach the finder
__version__ = getattr(_dxa, "__version__", "0.1")
