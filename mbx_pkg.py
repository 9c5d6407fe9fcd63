"""Import helper for the hyphenated package directory
`minibase-columnar-database_amd/` (registered as module `mbx_amd`)."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "minibase-columnar-database_amd")


def load():
    if "mbx_amd" in sys.modules:
        return sys.modules["mbx_amd"]
    spec = importlib.util.spec_from_file_location("mbx_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["mbx_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
