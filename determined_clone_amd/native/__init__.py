"""Native (C++) runtime components: scheduler and device detection."""
import importlib


def load():
    try:
        return importlib.import_module("determined_clone_amd.native._native")
    except ImportError:
        from determined_clone_amd.native import build

        build.build()
        return importlib.import_module("determined_clone_amd.native._native")
