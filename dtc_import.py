"""Import helper: the package directory `distributed-training-comparison_amd/` is not a valid
Python identifier, so it is imported by path and aliased as `dtc_amd`."""
import importlib
import os
import sys

PKG_DIR = "distributed-training-comparison_amd"


def load():
    if "dtc_amd" in sys.modules:
        return sys.modules["dtc_amd"]
    root = os.path.dirname(os.path.abspath(__file__))
    if root not in sys.path:
        sys.path.insert(0, root)
    return importlib.import_module(PKG_DIR)
