"""gatx — MI355X-native drop-in for loodvn/gat-pytorch's GATLayer hot path.

    from gatx import GATLayer          # == models/gat_layer.py:GATLayer, on libgatx.so (HIP)
    from gatx import GATModel          # layer stack wiring of models/GATModel.py (no Lightning)

Submodules `gatx.data`, `gatx.config`, `gatx.checkpoint`, `gatx.tuning` (the host path's explicit
switches; nothing is read from the environment) are pure Python/numpy. Everything that
computes (`GATLayer`, `GATModel`, `Graph`, `functional`) loads libgatx.so on first use and raises if
it is missing — there is no CPU fallback.
"""
__version__ = "0.1.0"

_LAZY = {
    "GATLayer": ("layer", "GATLayer"),
    "GATModel": ("model", "GATModel"),
    "Graph": ("graph", "Graph"),
    "clear_graph_cache": ("graph", "clear_graph_cache"),
    "gat_layer": ("functional", "gat_layer"),
}


_SUBMODULES = ("tuning", "config", "data", "checkpoint")


def __getattr__(name):
    if name in _SUBMODULES:
        import importlib
        return importlib.import_module(f"{__name__}.{name}")
    if name in _LAZY:
        import importlib
        mod, attr = _LAZY[name]
        return getattr(importlib.import_module(f"{__name__}.{mod}"), attr)
    raise AttributeError(name)
