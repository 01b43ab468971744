"""Host-side mirror of the UNC RT-DETR keypoint model's inference interface over
the HIP path in libspe.so:

    model = build_rtdetr(RtdetrConfig(depth=50))      # RTDETR(PResNet, HybridEncoder, RTDETRTransformer)
    model.load_state_dict(checkpoint["model"])         # the reference's state_dict keys
    out = model(images)                                # pred_logits / pred_pts / pred_sigmas (+ aux_outputs)
    results = RTDETRPostProcessor()(out, clip_bbox)    # [{logits, points, sigmas}] numpy, per image

Reference: UNC/src/zoo/rtdetr/rtdetr.py:20-53 (RTDETR.forward), rtdetr_decoder.py:672-710 (the
output dict in eval: the last layer's pred_logits / pred_pts / pred_sigmas and aux_outputs =
earlier decoder layers + the encoder top-k), rtdetr_postprocessor.py:44-76.  Every forward runs
the hand-written HIP kernels through the C ABI; there is no torch/CPU compute fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
from torch import nn

from . import _lib
from .misc import NestedTensor, nested_tensor_from_tensor_list
from .rtdetr_spec import RtdetrConfig, rtdetr_param_shapes, random_rtdetr_weights  # noqa: F401


class RTDETR(nn.Module):
    """RTDETR(PResNet-vd, HybridEncoder, RTDETRTransformer) with the sigma head, eval forward.
    dtype "bf16": bf16 storage / MFMA with fp32 accumulation, LayerNorm, softmax and heads;
    "fp32": exact-f32 MFMA everywhere (parity path)."""

    def __init__(self, cfg: RtdetrConfig, dtype: str = "bf16", aux_outputs: bool = True):
        super().__init__()
        self.cfg, self.dtype, self.aux_outputs = cfg, dtype, aux_outputs
        self.num_queries = cfg.num_queries
        self._pending = {}
        self._ready = False
        self._ws = {}
        c = _lib.RtdetrConfig(cfg.depth, cfg.input_size, cfg.num_queries, cfg.dec_layers, cfg.enc_ff, cfg.dec_ff,
                              cfg.csp_hidden, cfg.num_classes,
                              _lib.SPE_DTYPE_BF16 if dtype == "bf16" else _lib.SPE_DTYPE_F32)
        h = ctypes.c_void_p()
        L = _lib.lib()
        _lib.check(L.spe_rtdetr_create(ctypes.byref(c), ctypes.byref(h)), "spe_rtdetr_create")
        self._h = h
        self._keys = [L.spe_model_param_name(h, i).decode() for i in range(L.spe_model_num_params(h))]

    def param_keys(self):
        return list(self._keys)

    def load_state_dict(self, state_dict, strict: bool = True):
        """The reference's state_dict (torch tensors or numpy); BatchNorm num_batches_tracked
        buffers are ignored.  Returns (missing, unexpected) like nn.Module."""
        L = _lib.lib()
        unexpected = []
        for k, v in state_dict.items():
            if k.endswith("num_batches_tracked"):
                continue
            if k not in self._keys:
                unexpected.append(k)
                continue
            a = np.ascontiguousarray(v.detach().cpu().numpy() if torch.is_tensor(v) else v, dtype=np.float32)
            _lib.check(L.spe_model_set_param(self._h, k.encode(), a.ctypes.data_as(ctypes.c_void_p), a.size),
                       f"set_param({k})")
            self._pending[k] = True
        missing = [k for k in self._keys if k not in self._pending]
        if strict and (missing or unexpected):
            raise RuntimeError(f"load_state_dict: missing={missing[:5]}... unexpected={unexpected[:5]}...")
        if not self._ready and len(self._pending) == len(self._keys):
            _lib.check(L.spe_model_finalize(self._h), "spe_model_finalize")
            self._ready = True
        return missing, unexpected

    def workspace(self, B, device, stream=None):
        """Per-(device, stream) workspace, like DETR.workspace."""
        device = torch.device(device)
        s = stream if stream is not None else torch.cuda.current_stream(device)
        key = (device.index if device.index is not None else torch.cuda.current_device(), s.cuda_stream)
        ws = self._ws.get(key)
        if ws is None or ws[1] < B:
            nbytes = _lib.lib().spe_model_workspace_bytes(self._h, B)
            with torch.cuda.stream(s):
                self._ws[key] = ws = (torch.empty(int(nbytes), dtype=torch.uint8, device=device), B)
        return ws[0]

    def forward(self, samples, clip_bbox=None, stream=None, aux=None, return_hs=False):
        """rtdetr.py:36-53 in eval.  Returns pred_logits [B,Q,C+1], pred_pts [B,Q,2], pred_sigmas
        [B,Q,2] (raw) and, with aux, the reference's aux_outputs list.  Passing `clip_bbox`
        ([B,4] device) also runs the fused RTDETRPostProcessor: probs, points_px, sigmas.
        return_hs adds "hs" [B,Q,256], the last decoder layer's output (the heads' input)."""
        if not self._ready:
            raise RuntimeError("RTDETR: load_state_dict() with every parameter before forward()")
        aux = self.aux_outputs if aux is None else aux
        if isinstance(samples, (list, tuple)):
            samples = nested_tensor_from_tensor_list(list(samples))
        images = samples.tensors if isinstance(samples, NestedTensor) else samples
        if not images.is_cuda:
            raise RuntimeError("RTDETR (HIP) expects device tensors")
        images = images.contiguous().float()
        B, C3, H, W = images.shape
        S, Q, C = self.cfg.input_size, self.cfg.num_queries, self.cfg.num_classes + 1
        if C3 != 3 or H != S or W != S:
            raise ValueError(f"expected [B,3,{S},{S}] input, got {tuple(images.shape)}")
        dev = images.device
        f = dict(device=dev)
        out = {"pred_logits": torch.empty(B, Q, C, **f), "pred_pts": torch.empty(B, Q, 2, **f),
               "pred_sigmas": torch.empty(B, Q, 2, **f)}
        if clip_bbox is not None:
            clip_bbox = clip_bbox.to(device=dev, dtype=torch.float32).contiguous()
            out.update(probs=torch.empty(B, Q, C, **f), points_px=torch.empty(B, Q, 2, **f),
                       sigmas=torch.empty(B, Q, 2, **f))
        nl = self.cfg.dec_layers - 1
        if aux:
            al, ap, asg = torch.empty(nl, B, Q, C, **f), torch.empty(nl, B, Q, 2, **f), torch.empty(nl, B, Q, 2, **f)
            el, ep = torch.empty(B, Q, C, **f), torch.empty(B, Q, 2, **f)
            topk = torch.empty(B, Q, dtype=torch.int32, device=dev)
        else:
            al = ap = asg = el = ep = topk = None
        if return_hs:
            out["hs"] = torch.empty(B, Q, 256, **f)
        o = _lib.RtdetrOutputs(_lib.ptr(out["pred_logits"]), _lib.ptr(out["pred_pts"]), _lib.ptr(out["pred_sigmas"]),
                               _lib.ptr(clip_bbox), _lib.ptr(out.get("probs")), _lib.ptr(out.get("points_px")),
                               _lib.ptr(out.get("sigmas")), _lib.ptr(al), _lib.ptr(ap), _lib.ptr(asg), _lib.ptr(el),
                               _lib.ptr(ep), _lib.ptr(topk), _lib.ptr(out.get("hs")))
        ws = self.workspace(B, dev, stream)
        _lib.check(_lib.lib().spe_rtdetr_forward(self._h, _lib.stream_ptr(stream), _lib.ptr(images), B, _lib.ptr(ws),
                                                 ws.numel(), ctypes.byref(o)), "spe_rtdetr_forward")
        if aux:   # rtdetr_decoder.py:680-700: decoder layers first, the encoder top-k last
            out["aux_outputs"] = [{"pred_logits": al[i], "pred_pts": ap[i], "pred_sigmas": asg[i]} for i in range(nl)]
            out["aux_outputs"].append({"pred_logits": el, "pred_pts": ep})
            out["topk"] = topk
        return out

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                _lib.lib().spe_model_destroy(self._h)
                self._h = None
        except Exception:
            pass


class RTDETRPostProcessor(nn.Module):
    """UNC/src/zoo/rtdetr/rtdetr_postprocessor.py:44-76: softmax probabilities, crop ->
    image pixels, sigma = exp(pred_sigmas); returns numpy dicts per image like the reference.
    When the forward already ran the fused post-process (clip_bbox given) its device results are
    reused."""

    def __init__(self, num_classes=11, use_focal_loss=False, num_top_queries=30, remap_mscoco_category=False):
        super().__init__()
        self.num_classes, self.num_top_queries = num_classes, num_top_queries

    @torch.no_grad()
    def forward(self, outputs, clip_bbox):
        if "probs" in outputs:
            prob, pts, sig = outputs["probs"], outputs["points_px"], outputs["sigmas"]
        else:
            prob = torch.softmax(outputs["pred_logits"], -1)
            cb = torch.stack([torch.as_tensor(b, dtype=torch.float32) for b in clip_bbox]).to(prob.device)
            pts = outputs["pred_pts"].clone()
            pts[..., 0] = pts[..., 0] * (cb[:, 2:3] - cb[:, 0:1]) + cb[:, 0:1]
            pts[..., 1] = pts[..., 1] * (cb[:, 3:4] - cb[:, 1:2]) + cb[:, 1:2]
            sig = torch.exp(outputs["pred_sigmas"])
        prob, pts, sig = prob.cpu().numpy(), pts.cpu().numpy(), sig.cpu().numpy()
        return [{"logits": prob[i], "points": pts[i], "sigmas": sig[i]} for i in range(prob.shape[0])]


def build_rtdetr(cfg: RtdetrConfig = None, dtype: str = "bf16"):
    """(model, postprocessor) of a speed config (UNC/configs/rtdetr_speed/*.yml fields)."""
    cfg = cfg or RtdetrConfig()
    return RTDETR(cfg, dtype), RTDETRPostProcessor(cfg.num_classes, num_top_queries=cfg.num_queries)
