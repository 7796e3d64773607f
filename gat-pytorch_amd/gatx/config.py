"""Per-dataset model configuration, mirroring the reference's `run_config.py`.

`data_config` restates `run_config.py:17-98` (treated as canonical); `LayerType`
restates `run_config.py:4-6`. `NOTEBOOK_VARIANTS` records where `Reproduce_Experiments.ipynb`
drifts from it (PPI skip/batch at ipynb:570-574, PATTERN batch at ipynb:690).
"""
from enum import Enum


class LayerType(Enum):
    GATLayer = 1
    PyTorch_Geometric = 2


class Dataset(Enum):
    PPI = 1
    Cora = 2
    Citeseer = 3
    Pubmed = 4


def _cfg(in_f, heads, concat, widths, classes, skip, dropout, l2, lr, batch):
    return {
        "layer_type": LayerType.GATLayer,
        "num_input_node_features": in_f,
        "num_layers": len(heads),
        "num_heads_per_layer": list(heads),
        "heads_concat_per_layer": list(concat),
        "head_output_features_per_layer": list(widths),
        "num_classes": classes,
        "add_skip_connection": list(skip),
        "dropout": dropout,
        "l2_reg": l2,
        "learning_rate": lr,
        "batch_size": batch,
        "num_epochs": 1000,
        "const_attention": False,
    }


data_config = {
    "PPI": _cfg(50, [4, 4, 6], [True, True, False], [50, 256, 256, 121], 121,
                [False, True, False], 0.0, 0.0, 0.005, 2),
    "PATTERN": _cfg(3, [4, 4, 4, 1], [True, True, True, False], [3, 12, 24, 12, 1], 1,
                    [True, True, True, True], 0, 0, 0.005, 8),
    "Cora": _cfg(1433, [8, 1], [True, False], [1433, 8, 7], 7, [False, False], 0.6, 0.0005,
                 0.005, 1),
    "Citeseer": _cfg(3703, [8, 1], [True, False], [3703, 8, 6], 6, [False, False], 0.6, 0.0005,
                     0.005, 1),
    "Pubmed": _cfg(500, [8, 8], [True, False], [500, 8, 3], 3, [False, False], 0.6, 0.001,
                   0.01, 1),
}

NOTEBOOK_VARIANTS = {
    "PPI": {"add_skip_connection": [True, True, True], "batch_size": 1},
    "PATTERN": {"batch_size": 32},
}
