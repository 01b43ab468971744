"""ctypes binding of libspe.so (C ABI in include/spe.h).

torch is imported first on purpose: its bundled libamdhip64.so.7 is then the HIP runtime the
library binds to (same SONAME), so device pointers and streams are shared with torch.
There is no fallback: if the library is missing the import fails loudly.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

# HIP graph capture of this library's launches (PosePipeline(use_graph=True)) replays correctly
# only with the ROCm runtime's graph packet capture off: with it on, a replay issued after the
# stream has synchronised reads wrong kernel arguments (measured: the first replay is exact, the
# later ones are not).  The runtime reads the switch when HIP initialises and
# it applies to every graph of the process, so importing spe does not set it: a caller that wants
# graph capture sets DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 before its first device call (tests/conftest.py
# does), or opts in with SPE_GRAPH_CAPTURE=1 before importing spe.  The pipeline verifies its
# captured graph against eager execution either way and raises if they differ.
if os.environ.get("SPE_GRAPH_CAPTURE") == "1":
    os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SPE_LIB_PATH") or os.path.join(_HERE, "libspe.so")   # override: kernel A/B builds

# the include/spe.h version this binding is written against: any other library is refused, including
# one named by SPE_LIB_PATH (an A/B build of an older tree would otherwise be called with this
# binding's argument lists)
ABI_VERSION = 9

P = ctypes.c_void_p
I = ctypes.c_int
I64 = ctypes.c_int64
F = ctypes.c_float
D = ctypes.c_double

SPE_DTYPE_BF16, SPE_DTYPE_F32, SPE_DTYPE_F16, SPE_DTYPE_F32X3, SPE_DTYPE_F32X6, SPE_DTYPE_F32H3 = 0, 1, 2, 4, 5, 6
SPE_STAGE_ENCODE, SPE_STAGE_DECODE, SPE_STAGE_BACKBONE, SPE_STAGE_TRANSFORMER = 1, 2, 4, 8
SPE_PNP_EPNP, SPE_PNP_RANSAC_P3P_LM, SPE_PNP_EPNP_RANSAC_SIGMA, SPE_PNP_EPNP_LM, SPE_PNP_EPNP_CERES = 0, 1, 2, 3, 4
SPE_PNP_OK, SPE_PNP_NO_FG, SPE_PNP_CV_ERROR, SPE_PNP_RANSAC_FALLBACK, SPE_PNP_UNPINNED = 0, 1, 2, 3, 4

# every symbol include/spe.h declares (checked by tests/test_capi.py)
EXPORTS = ["spe_abi_version", "spe_last_error", "spe_model_create", "spe_model_destroy", "spe_model_set_param",
           "spe_model_num_params", "spe_model_param_name", "spe_model_finalize", "spe_model_workspace_bytes",
           "spe_forward", "spe_forward_stages", "spe_forward_stages_u8", "spe_preprocess", "spe_criterion", "spe_ensemble_fuse", "spe_postprocess", "spe_pnp_batch", "spe_self_assess", "spe_speed_score", "spe_model_profile_begin",
           "spe_model_profile_end", "spe_model_profile_get", "spe_debug_gemm", "spe_debug_gemm_path", "spe_debug_gemm_h3", "spe_debug_ffn_h3", "spe_debug_ffn_h3_perm", "spe_debug_gemm_planes", "spe_debug_attention",
           "spe_debug_layernorm", "spe_debug_ffn", "spe_debug_xattn", "spe_debug_xattn_h3", "spe_debug_upconv", "spe_debug_btail", "spe_debug_decsa", "spe_debug_decproj", "spe_debug_decxproj", "spe_debug_wfrag_pack", "spe_debug_decffn", "spe_debug_decq", "spe_debug_btail_perm", "spe_debug_stempool", "spe_rtdetr_create", "spe_rtdetr_forward",
           "spe_jpeg_workspace_bytes", "spe_jpeg_decode"]


class ModelConfig(ctypes.Structure):
    _fields_ = [("input_size", I), ("num_queries", I), ("enc_layers", I), ("dec_layers", I), ("hidden_dim", I),
                ("nheads", I), ("dim_feedforward", I), ("sigma_head", I), ("dtype", I),
                ("attn_dtype", I)]


class ForwardOutputs(ctypes.Structure):
    _fields_ = [("logits", P), ("points", P), ("clip_bbox", P), ("probs", P), ("points_px", P),
                ("log_sigmas", P), ("sigmas", P), ("hs", P), ("aux_logits", P), ("aux_points", P)]


class RtdetrConfig(ctypes.Structure):
    _fields_ = [("depth", I), ("input_size", I), ("num_queries", I), ("dec_layers", I), ("enc_ff", I), ("dec_ff", I),
                ("csp_hidden", I), ("num_classes", I), ("dtype", I)]


class RtdetrOutputs(ctypes.Structure):
    _fields_ = [("logits", P), ("points", P), ("log_sigmas", P), ("clip_bbox", P), ("probs", P), ("points_px", P),
                ("sigmas", P), ("aux_logits", P), ("aux_points", P), ("aux_log_sigmas", P), ("enc_logits", P),
                ("enc_points", P), ("topk", P), ("hs", P)]


class SpeError(RuntimeError):
    pass


_lib = None


def load(path: str):
    """CDLL of `path` with the argument types bound; ImportError unless it is ABI_VERSION's library."""
    if not os.path.exists(path):
        raise ImportError(f"libspe.so not built ({path}); run __graft_entry__.build()")
    L = ctypes.CDLL(path)
    if not hasattr(L, "spe_abi_version"):
        raise ImportError(f"{path} exports no spe_abi_version")
    L.spe_abi_version.restype = I
    v = L.spe_abi_version()
    if v != ABI_VERSION:
        raise ImportError(f"{path}: ABI version {v}, this binding needs {ABI_VERSION}")
    L.spe_last_error.restype = ctypes.c_char_p
    L.spe_model_create.argtypes = [ctypes.POINTER(ModelConfig), ctypes.POINTER(P)]
    L.spe_model_destroy.argtypes = [P]
    L.spe_model_destroy.restype = None
    L.spe_model_set_param.argtypes = [P, ctypes.c_char_p, P, I64]
    L.spe_model_num_params.argtypes = [P]
    L.spe_model_param_name.argtypes = [P, I]
    L.spe_model_param_name.restype = ctypes.c_char_p
    L.spe_model_finalize.argtypes = [P]
    L.spe_model_workspace_bytes.argtypes = [P, I]
    L.spe_model_workspace_bytes.restype = I64
    L.spe_forward.argtypes = [P, P, P, I, P, I64, ctypes.POINTER(ForwardOutputs)]
    L.spe_forward_stages.argtypes = [P, P, P, I, P, I64, ctypes.POINTER(ForwardOutputs), I]
    L.spe_forward_stages_u8.argtypes = [P, P, P, I, I, P, I64, ctypes.POINTER(ForwardOutputs), I]
    L.spe_postprocess.argtypes = [P, P, P, P, I, I, P, P]
    L.spe_preprocess.argtypes = [P, P, I, I, I, I, P, I, P, P, P]
    L.spe_ensemble_fuse.argtypes = [P, P, P, I, I, I, I, P, P]
    L.spe_criterion.argtypes = [P, P, P, P, P, I, I, I, I, I, F, F, F, D, P, P]
    L.spe_pnp_batch.argtypes = [P, P, P, P, I, I, I, P, P, I, F, I, D, P, P, P, P, P, P, P, P]
    L.spe_speed_score.argtypes = [P, P, P, P, P, I, P, P]
    L.spe_self_assess.argtypes = [P, P, P, P, P, P, I, I, I, F, F, I, P, P, P]
    L.spe_model_profile_begin.argtypes = [P, ctypes.c_char_p]
    L.spe_model_profile_end.argtypes = [P]
    L.spe_model_profile_get.argtypes = [P, I, ctypes.c_char_p, I, ctypes.POINTER(D), ctypes.POINTER(D),
                                        ctypes.POINTER(D)]
    L.spe_debug_gemm.argtypes = [P, I, I, P, I, P, I, I] + [I] * 7 + [P, I, I, I, I, P, P, I, I, P, I, I, I, I, I, P, P, I]
    L.spe_debug_gemm_path.argtypes = []
    L.spe_debug_gemm_h3.argtypes = [P, I, P, I] + [I] * 7 + [I, I, I, I, P, P, I, I, P, I, P, I, P, P, P, ctypes.c_float]
    L.spe_debug_ffn_h3.argtypes = [P, P, I, P, I, I, I, P, I, P, P, I, P, P, P, P, P, ctypes.c_float]
    L.spe_debug_ffn_h3_perm.argtypes = [I]
    L.spe_debug_gemm_planes.argtypes = [P, I, I, P, I, P, I, I] + [I] * 7 + [P, I, I, I, I, P, P, I, I, P, I, P, I]
    L.spe_debug_attention.argtypes = [P, I, P, I, P, I, P, P, I, I, I, I, I, F]
    L.spe_debug_layernorm.argtypes = [P, I, P, P, P, P, P, I, I]
    L.spe_debug_ffn.argtypes = [P, P, I, P, I, P, P, I, P, P, P, P, I, I, I, I, P, I]
    L.spe_debug_xattn.argtypes = [P, P, I, P, I, P, I, P, I, P, P, P, I, I, I, I, I, P]
    L.spe_debug_xattn_h3.argtypes = [P, P, I, P, P, P, P, P, P, I, P, I, I, I, I, P, P]
    L.spe_debug_upconv.argtypes = [P, I, P, P, I, I, I, I, I]
    L.spe_debug_btail.argtypes = [P, P, I, I, P, P, I, P, P, P, I, P, P, I, I]
    L.spe_debug_btail_perm.argtypes = [I]
    L.spe_debug_decsa.argtypes = [P, P, I, I, I, P, I, P, P, I, P, P, P, I, P, P, P, ctypes.c_float]
    L.spe_debug_decproj.argtypes = [P, P, I, P, I, I, I, P, I, P, P, P]
    L.spe_debug_wfrag_pack.argtypes = [P, P, I, I, P]
    L.spe_debug_decffn.argtypes = [P, P, I, I, I, P, I, P, P, I, P, P, P, P, I, P]
    L.spe_debug_decq.argtypes = [P, P, I, I, I, P, I, P, P, I, I, P, I]
    L.spe_debug_decxproj.argtypes = [P, P, I, P, I, I, I, I, P, I, P, P, I, P, P, P]
    L.spe_debug_stempool.argtypes = [P, P, P, I, P, P, I, I, I]
    L.spe_rtdetr_create.argtypes = [ctypes.POINTER(RtdetrConfig), ctypes.POINTER(P)]
    L.spe_rtdetr_forward.argtypes = [P, P, P, I, P, I64, ctypes.POINTER(RtdetrOutputs)]
    L.spe_jpeg_workspace_bytes.argtypes = [I, I, I, I64]
    L.spe_jpeg_workspace_bytes.restype = I64
    L.spe_jpeg_decode.argtypes = [P, P, P, P, I, I, I, I64, P, P, P, I64]
    return L


def lib():
    global _lib
    if _lib is None:
        _lib = load(LIB_PATH)
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().spe_last_error().decode(errors="replace")
        raise SpeError(f"{what} failed with code {rc}: {msg}")


def ptr(t):
    """Device (or host) pointer of a torch tensor, None for None."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)
