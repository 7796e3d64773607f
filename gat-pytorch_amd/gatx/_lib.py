"""ctypes binding of libgatx.so (the C-ABI declared in include/gatx.h).

torch is imported first so that torch's own HIP runtime (soname libamdhip64.so.7) is the one the
library binds to: device pointers, streams and the caching allocator are then shared. There is no
CPU fallback: if the library is missing the import fails loudly (build it with
`make -C gat-pytorch_amd/csrc` or `python -c "import __graft_entry__ as g; g.build()"`).
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL: shares torch's libamdhip64)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GATX_LIB", os.path.join(_HERE, "libgatx.so"))

ARGMAX_CAP = 1024  # GATX_ARGMAX_CAP
META_WORDS = 520   # GATX_META_WORDS

c_i = ctypes.c_int
c_i64 = ctypes.c_int64
c_u64 = ctypes.c_uint64
c_f = ctypes.c_float
c_sz = ctypes.c_size_t
P = ctypes.c_void_p

# name: (restype, argtypes) — mirrors include/gatx.h one-to-one
SIGNATURES = {
    "gatx_last_error": (ctypes.c_char_p, []),
    "gatx_version": (c_i, []),
    "gatx_region_mark": (c_i, [ctypes.c_uint32, P]),
    "gatx_graph_meta_workspace_bytes": (c_sz, []),
    "gatx_graph_meta": (c_i, [P, c_i, c_i64, c_i64, c_i, c_i64, P, P, P]),
    "gatx_graph_build_workspace_bytes": (c_sz, [c_i64, c_i64, c_i64]),
    "gatx_graph_build": (c_i, [P, c_i, c_i64, c_i64, c_i, c_i64, c_i64, P, P, P, P, P, P, P,
                               c_sz, P]),
    "gatx_graph_transpose_workspace_bytes": (c_sz, [c_i64, c_i64]),
    "gatx_graph_transpose": (c_i, [P, P, c_i64, c_i64, P, P, P, P, P, c_sz, P]),
    "gatx_prepare_weights": (c_i, [P, P, c_i, c_i, c_i64, P, P]),
    "gatx_prepare_weights_floats": (c_i64, [c_i, c_i, c_i64, c_i]),
    "gatx_gemm_f32": (c_i, [c_i64, c_i64, c_i64, P, c_i64, c_i64, P, c_i64, c_i64, P, c_i64,
                            c_i64, P, c_i64, c_i, P, c_sz, P]),
    "gatx_gemm_workspace_bytes": (c_sz, [c_i64, c_i64, c_i64]),
    "gatx_transpose_f32": (c_i, [c_i64, c_i64, P, c_i64, P, c_i64, P]),
    "gatx_gemm_f32_batched": (c_i, [c_i64, c_i64, c_i64, c_i64, P, c_i64, c_i64, c_i64, P,
                                    c_i64, c_i64, c_i64, P, c_i64, c_i64, c_i, P, c_i64, P, c_i64,
                                    c_i64, c_i, P]),
    "gatx_edge_forward_ex": (c_i, [P, c_i64, c_i64, P, P, P, P, P, c_i64, c_i, c_i, c_i, c_i, c_i,
                                   c_i, c_i, c_i, P, c_f, P, P, c_i64, P, c_i64, c_i, P, c_i64,
                                   P]),
    "gatx_edge_forward_hubs": (c_i, [P, c_i64, c_i64, P, P, P, P, P, c_i64, c_i, c_i, c_i, c_i,
                                     c_i, c_i, c_i, c_i, P, c_f, P, P, c_i64, P, c_i64, c_i, P,
                                     c_i64, c_i, P, P, c_i64, P, P]),
    "gatx_edge_forward_drop": (c_i, [P, c_i64, c_i64, P, P, P, P, P, c_i64, c_i, c_i, c_i, c_i,
                                     c_i, c_i, c_i, c_i, P, c_f, P, P, c_i64, P, c_i64, c_i, P,
                                     c_i64, c_i, P, P, c_i64, P, c_f, P, P]),
    "gatx_edge_forward_skip": (c_i, [P, c_i64, c_i64, P, P, P, P, P, c_i64, c_i, c_i, c_i, c_i,
                                     c_i, c_i, c_i, c_i, P, c_f, P, P, c_i64, P, c_i64, c_i, P,
                                     c_i64, c_i, P, P, c_i64, P, c_f, P, P, P]),
    "gatx_edge_forward_hub_part_bytes": (c_sz, [c_i64, c_i, c_i, c_i, c_i]),
    "gatx_graph_hub_bound": (c_i64, [c_i64, c_i]),
    "gatx_graph_hub_plan": (c_i, [P, c_i64, c_i, P, c_i64, P, P]),
    "gatx_graph_segments_workspace_bytes": (c_sz, [c_i64]),
    "gatx_graph_segments": (c_i, [P, P, c_i64, c_i, P, P, P, c_sz, P]),
    "gatx_graph_segments_max": (c_i, []),
    "gatx_edge_lds_rows": (c_i, []),
    "gatx_edge_records_src": (c_i, [P, P, P, P, P, P, P, c_i64, c_i64, c_i, c_i, c_f, P, P, P, c_i64,
                                    c_i64, P, P]),
    "gatx_edge_records": (c_i, [P, P, P, P, P, c_i64, c_i64, c_i, c_i, c_f, P, P, P, P, P, P]),
    "gatx_edge_lds_forward": (c_i, [P, c_i64, P, c_i64, P, c_i64, P, P, c_i64, c_i, c_i, P, P, c_i64,
                                    P, c_i64, c_i, c_f, P, P]),
    "gatx_edge_lds_mean_forward": (c_i, [P, c_i64, P, c_i64, P, c_i64, P, P, c_i64, c_i, c_i, P, P,
                                         c_i64, P, c_i64, c_i, c_f, P, P]),
    "gatx_pad_rows": (c_i, [P, c_i64, c_i64, c_i64, P, c_i64, P]),
    "gatx_projection_gemm": (c_i, [c_i64, c_i64, c_i64, P, c_i64, c_i64, P, c_i64, c_i64, P,
                                   c_i64, c_i64, P, c_i64, P, c_sz, P]),
    "gatx_projection_scores_workspace_bytes": (c_sz, [c_i64, c_i64, c_i64, c_i]),
    "gatx_projection_gemm_scores": (c_i, [c_i64, c_i64, c_i64, P, c_i64, c_i64, P, c_i64, c_i64,
                                          P, c_i64, P, c_i, c_i, P, P, c_sz, P]),
    "gatx_projection_gemm3": (c_i, [c_i64, c_i64, c_i64, P, c_i64, c_i64, P, c_i64, c_i64, P,
                                    c_i64, c_i64, P, c_i64, c_i64, P, c_i64, P, c_sz, P]),
    "gatx_prepare_weights_skip": (c_i, [P, P, c_i, c_i, c_i64, P, c_i, c_i64, P, P]),
    "gatx_prepare_weights_skip_floats": (c_i64, [c_i, c_i, c_i64, c_i, c_i64]),
    "gatx_prepare_go_ex": (c_i, [P, P, c_i64, c_i, c_i, c_i, c_i, P, P, c_i64, c_f, P, P]),
    "gatx_dropout": (c_i, [P, c_i64, c_f, P, P, P]),
    "gatx_skip_weight_grad": (c_i, [P, c_i, c_i64, c_i64, P, P]),
    "gatx_set_debug": (None, [c_i]),
    "gatx_set_gemm_mode": (None, [c_i]),
    "gatx_get_gemm_mode": (c_i, []),
    "gatx_gemm_fallback_read": (c_i, [P, c_i, P]),
    "gatx_gemm_layout_mode": (c_i, [c_i, c_i]),
    "gatx_weight_planes_bytes": (c_sz, [c_i64, c_i64]),
    "gatx_weight_planes": (c_i, [P, c_i64, c_i64, c_i64, P, P]),
    "gatx_gemm_planes": (c_i, [c_i64, c_i64, c_i64, P, c_i64, P, c_i64, P, P, c_i64, c_i64, P,
                               c_i64, c_i64, P, c_i64, c_i, P, c_i, c_i, P, c_i, P, P, c_sz, P]),
    "gatx_absmax_rows_cols": (c_i, [P, c_i64, c_i64, c_i64, P, P, P]),
    "gatx_gemm_wgrad": (c_i, [c_i64, c_i64, c_i64, P, c_i64, P, c_i64, P, P, c_i64, P, c_sz, P]),
    "gatx_gemm_splitk_workspace_bytes": (c_sz, [c_i64, c_i64, c_i64]),
    "gatx_gemm_f32_splitk": (c_i, [c_i64, c_i64, c_i64, P, c_i64, c_i64, P, c_i64, c_i64, P, c_i64,
                                   c_i, P, c_sz, P]),
    "gatx_node_scores": (c_i, [P, c_i64, c_i, c_i, P, P, P]),
    "gatx_attention_max_workspace_bytes": (c_sz, []),
    "gatx_attention_max": (c_i, [P, P, c_i64, P, P, c_i, P, P, P, P]),
    "gatx_edge_forward": (c_i, [P, P, P, P, P, P, P, c_i64, c_i64, c_i, c_i, c_i, c_i, P, c_f,
                                P, P, P, P, P, P]),
    "gatx_attention_alpha": (c_i, [P, P, P, c_i64, P, P, P, c_i, c_i, P, P, P]),
    "gatx_attention_alpha_ei": (c_i, [P, c_i, c_i64, c_i64, P, P, P, P, c_i, c_i, P, P, P, P,
                                      P]),
    "gatx_prepare_go": (c_i, [P, P, c_i64, c_i, c_i, c_i, c_i, P, P, P]),
    "gatx_edge_backward_dst": (c_i, [P, P, P, P, P, P, P, c_i64, c_i64, c_i, c_i, c_i, c_f, P,
                                     P, P, P, P, P, c_i64, P]),
    "gatx_edge_backward_dst_ex": (c_i, [P, c_i64, c_i64, P, P, P, P, P, P, c_i64, c_i64, c_i,
                                        c_i, P, c_i64, c_i64, c_f, P, P, P, P, P, c_i64,
                                        c_i64, P]),
    "gatx_edge_backward_hub_part_bytes": (c_sz, [c_i64, c_i, c_i, c_i]),
    "gatx_edge_backward_dst_hubs": (c_i, [P, c_i64, c_i64, P, P, P, P, P, P, c_i64, c_i64, c_i,
                                          c_i, P, c_i64, c_i64, c_f, P, P, P, P, P, c_i64,
                                          c_i64, c_i, P, P, c_i64, P, P]),
    "gatx_edge_backward_src_hubs": (c_i, [P, P, P, P, P, P, P, c_i64, c_i64, c_i, c_i, c_i, c_i,
                                          c_f, P, P, P, P, P, c_i64, c_i, P, P, c_i64, P, P]),
    "gatx_edge_backward_src_scores": (c_i, [P, P, c_i64, c_i64, c_i, P, P, P, c_i64, c_i64, P]),
    "gatx_gemm_splitk_batched_workspace_bytes": (c_sz, [c_i64, c_i64, c_i64, c_i64]),
    "gatx_gemm_f32_splitk_batched": (c_i, [c_i64, c_i64, c_i64, c_i64, P, c_i64, c_i64, c_i64, P,
                                           c_i64, c_i64, c_i64, P, c_i64, c_i64, c_i, P, c_sz,
                                           P]),
    "gatx_max_backward_workspace_bytes": (c_sz, []),
    "gatx_max_backward": (c_i, [P, P, P, P, P, P, c_i64, c_i64, P, c_i, P, P, c_i64, c_i64, P,
                                P]),
    "gatx_edge_backward_src": (c_i, [P, P, P, P, P, P, P, c_i64, c_i64, c_i, c_i, c_i, c_i, c_f,
                                     P, P, P, P, P, c_i64, P]),
    "gatx_weight_grads": (c_i, [P, P, P, c_i, c_i, c_i64, P, P, P]),
    "gatx_colsum": (c_i, [P, c_i64, c_i64, c_i64, P, P]),
    "gatx_bce_logits_workspace_bytes": (c_sz, []),
    "gatx_bce_logits": (c_i, [P, P, c_i64, c_f, P, P, P, P]),
    "gatx_scale_by_scalar": (c_i, [P, P, c_i64, P, P]),
    "gatx_attention_norm_workspace_bytes": (c_sz, []),
    "gatx_attention_norm": (c_i, [P, c_i64, c_i, P, c_i, P, c_f, c_i, P, P, P]),
    "gatx_attention_norm_backward": (c_i, [P, c_i64, c_i, P, c_i, P, P, c_f, P, P]),
    "gatx_attention_norm_multi_workspace_bytes": (c_sz, [c_i]),
    "gatx_attention_norm_multi": (c_i, [P, P, c_i, c_i64, P, c_i, P, c_f, P, P, P]),
}


class GatxError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"gatx: HIP library not found at {LIB_PATH}. The GAT hot path has no CPU fallback; "
            "build it with `make -C gat-pytorch_amd/csrc` (hipcc --offload-arch=gfx950).")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib.gatx_last_error().decode(errors="replace")
        raise GatxError(f"gatx {what} failed (code {rc}): {msg}")


def ptr(t) -> int | None:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def version(t) -> int:
    """In-place version counter of a tensor for cache keys. Inference tensors (made under
    torch.inference_mode) track none and cannot be modified in place outside it: 0."""
    return 0 if t.is_inference() else t._version


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def call(name: str, *args):
    check(getattr(lib, name)(*args), name)
