"""Import shim: the package source lives in ``./hybrid-rag-colbertv2_amd/``.

A hyphenated directory is not an importable Python name, so this module loads
that directory as the package ``hybrid_rag_colbertv2_amd`` and replaces itself
in ``sys.modules``.  ``import hybrid_rag_colbertv2_amd`` (and its submodules)
then work from the repository root.
"""
import importlib.util
import os
import sys

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hybrid-rag-colbertv2_amd")
_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(_DIR, "__init__.py"), submodule_search_locations=[_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
