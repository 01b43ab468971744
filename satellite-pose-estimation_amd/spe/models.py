"""Host-side mirror of the reference model interface (REV/models/__init__.py:5-6,
REV/models/detr_speed.py:32-100,264-336) over the HIP path in libspe.so.

    model, criterion, postprocessors = build_model(args)
    model.load_state_dict(state_dict)      # the reference's 412 keys (checkpoint['model'])
    out = model(samples)                   # NestedTensor | list[Tensor] | Tensor [B,3,S,S]
    results = postprocessors['points'](out, clip_bbox_list)

Every forward runs the hand-written HIP kernels through the C ABI; there is no torch/CPU
compute fallback.  torch is only used for device memory and the current stream.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
from torch import nn

from . import _lib
from .config import SpeConfig
from .misc import NestedTensor, nested_tensor_from_tensor_list


class DETR(nn.Module):
    """Keypoint-set predictor (REV/models/detr_speed.py:32-100), HIP implementation.

    dtype "bf16": bf16 storage / MFMA with fp32 accumulation, softmax, LayerNorm and heads
    (throughput path).  dtype "fp32": exact-f32 MFMA everywhere (parity path).  dtype "fp32x3":
    the fp32 model with split-bf16 MFMA compute (every fp32 operand x = hi + lo in bf16, products
    hi.hi + hi.lo + lo.hi, fp32 accumulation; fast parity path).  dtype "fp32x6": the accuracy-contract
    mode -- fp32x3's attention, every GEMM / convolution at near-fp32 precision (three-way split,
    six products).  dtype "fp32h3": fp32x6 with the backbone / encoder GEMMs and
    convolutions as three fp16 MFMAs on a power-of-two-scaled two-way fp16 split (the same
    near-fp32 products at half fp32x6's MFMAs).
    attn_dtype "fp16" (bf16 models): the encoder self-attention's q/k/V operands are stored
    and multiplied in fp16 (BASELINE config 5, "fp16 MFMA attention")."""

    def __init__(self, cfg: SpeConfig, dtype: str = "bf16", aux_loss: bool = False, attn_dtype: str = None):
        super().__init__()
        self.cfg = cfg
        self.num_queries = cfg.num_queries
        self.aux_loss = aux_loss
        self.dtype = dtype
        if attn_dtype not in (None, dtype, "fp16") or (attn_dtype == "fp16" and dtype != "bf16"):
            raise ValueError(f"attn_dtype {attn_dtype!r}: None, the model dtype, or 'fp16' for bf16 models")
        self.attn_dtype = attn_dtype or dtype
        self._pending = {}
        self._handle = None
        self._ws = {}          # (device, stream) -> (workspace, batch it was sized for)
        L = _lib.lib()
        c = _lib.ModelConfig(cfg.input_size, cfg.num_queries, cfg.enc_layers, cfg.dec_layers, cfg.hidden_dim,
                             cfg.nheads, cfg.dim_feedforward, int(cfg.sigma_head),
                             {"bf16": _lib.SPE_DTYPE_BF16, "fp32": _lib.SPE_DTYPE_F32,
                              "fp32x3": _lib.SPE_DTYPE_F32X3, "fp32x6": _lib.SPE_DTYPE_F32X6,
                              "fp32h3": _lib.SPE_DTYPE_F32H3}[dtype],
                             _lib.SPE_DTYPE_F16 if self.attn_dtype == "fp16" else 0)
        h = ctypes.c_void_p()
        _lib.check(L.spe_model_create(ctypes.byref(c), ctypes.byref(h)), "spe_model_create")
        self._h = h
        self._keys = [L.spe_model_param_name(h, i).decode() for i in range(L.spe_model_num_params(h))]

    # ---------------------------------------------------------------- parameters
    def param_keys(self):
        return list(self._keys)

    def load_state_dict(self, state_dict, strict: bool = True):
        """Accepts the reference's state_dict (torch tensors or numpy arrays).  Keys outside the
        inference path (none for REV) are reported as unexpected, like nn.Module."""
        L = _lib.lib()
        unexpected = []
        for k, v in state_dict.items():
            if k.endswith("num_batches_tracked"):       # FrozenBatchNorm2d drops it (backbone.py:36-42)
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
        self._finalize()
        return missing, unexpected

    def _finalize(self):
        if self._handle is None and len(self._pending) == len(self._keys):
            _lib.check(_lib.lib().spe_model_finalize(self._h), "spe_model_finalize")
            self._handle = self._h

    def workspace(self, B, device, stream=None):
        """The default workspace of forward() on `stream` (the current stream if None): one per
        (device, stream), so forwards issued on different streams never share intermediates;
        forwards on one stream are ordered by it.  Allocated from torch's caching allocator on
        that stream, so a regrown workspace's old block is only reused in stream order."""
        device = torch.device(device)
        s = stream if stream is not None else torch.cuda.current_stream(device)
        key = (device.index if device.index is not None else torch.cuda.current_device(), s.cuda_stream)
        ws = self._ws.get(key)
        if ws is None or ws[1] < B:
            nbytes = _lib.lib().spe_model_workspace_bytes(self._h, B)
            with torch.cuda.stream(s):
                self._ws[key] = ws = (torch.empty(int(nbytes), dtype=torch.uint8, device=device), B)
        return ws[0]

    def new_workspace(self, B, device):
        """A separate workspace for another in-flight batch (encode/decode overlap)."""
        return torch.empty(int(_lib.lib().spe_model_workspace_bytes(self._h, B)), dtype=torch.uint8, device=device)

    # ---------------------------------------------------------------- forward
    def _outputs(self, B, dev, clip_bbox, return_hs):
        Q = self.cfg.num_queries
        out = {"pred_logits": torch.empty(B, Q, 12, device=dev), "pred_points": torch.empty(B, Q, 2, device=dev)}
        if self.cfg.sigma_head:
            out["pred_sigmas"] = torch.empty(B, Q, 2, device=dev)
            out["sigmas"] = torch.empty(B, Q, 2, device=dev)
        if return_hs:
            out["hs"] = torch.empty(B, Q, self.cfg.hidden_dim, device=dev)
        if clip_bbox is not None:
            out["probs"] = torch.empty(B, Q, 12, device=dev)
            out["points_px"] = torch.empty(B, Q, 2, device=dev)
        aux_l = aux_p = None
        if self.aux_loss and self.cfg.dec_layers > 1:       # REV/models/detr_speed.py:88-99
            aux_l = torch.empty(self.cfg.dec_layers - 1, B, Q, 12, device=dev)
            aux_p = torch.empty(self.cfg.dec_layers - 1, B, Q, 2, device=dev)
            out["aux_outputs"] = [{"pred_logits": a, "pred_points": p} for a, p in zip(aux_l, aux_p)]
        o = _lib.ForwardOutputs(_lib.ptr(out["pred_logits"]), _lib.ptr(out["pred_points"]), _lib.ptr(clip_bbox),
                                _lib.ptr(out.get("probs")), _lib.ptr(out.get("points_px")),
                                _lib.ptr(out.get("pred_sigmas")), _lib.ptr(out.get("sigmas")),
                                _lib.ptr(out.get("hs")), _lib.ptr(aux_l), _lib.ptr(aux_p))
        return out, o

    def encode(self, images, ws, stream=None, part=None, B=None):
        """Encode stage (backbone, neck, input_proj, encoder): images -> memory kept in `ws`.
        part="backbone": up to input_proj (images -> src in `ws`); part="transformer": the
        encoder layers over the src a backbone part left in `ws` (images may be None, B given)."""
        stage = {None: _lib.SPE_STAGE_ENCODE, "backbone": _lib.SPE_STAGE_BACKBONE,
                 "transformer": _lib.SPE_STAGE_TRANSFORMER}[part]
        B = images.shape[0] if images is not None else int(B)
        if images is not None and images.dtype == torch.uint8:
            ch = self._crop_channels(images)
            _lib.check(_lib.lib().spe_forward_stages_u8(self._h, _lib.stream_ptr(stream), _lib.ptr(images), ch, B,
                                                        _lib.ptr(ws), ws.numel(), None, stage), "spe_forward_stages_u8")
            return
        _lib.check(_lib.lib().spe_forward_stages(self._h, _lib.stream_ptr(stream), _lib.ptr(images), B, _lib.ptr(ws),
                                                 ws.numel(), None, stage), "spe_forward_stages")

    def _crop_channels(self, crops):
        """8-bit crops [B,S,S] (grayscale) or [B,S,S,3] (RGB), contiguous on the device -> channels."""
        S = self.cfg.input_size
        if not crops.is_cuda or not crops.is_contiguous():
            raise ValueError("u8 crops: a contiguous device tensor")
        if crops.dim() == 3 and tuple(crops.shape[1:]) == (S, S):
            return 1
        if crops.dim() == 4 and tuple(crops.shape[1:]) == (S, S, 3):
            return 3
        raise ValueError(f"u8 crops: expected [B,{S},{S}] or [B,{S},{S},3], got {tuple(crops.shape)}")

    def decode(self, B, ws, clip_bbox=None, stream=None, return_hs=False):
        """Decode stage (decoder, heads, fused PostProcess) of the memory an encode() left in `ws`."""
        dev = ws.device
        if clip_bbox is not None:
            clip_bbox = clip_bbox.to(device=dev, dtype=torch.float32).contiguous()
        out, o = self._outputs(B, dev, clip_bbox, return_hs)
        _lib.check(_lib.lib().spe_forward_stages(self._h, _lib.stream_ptr(stream), None, B, _lib.ptr(ws), ws.numel(),
                                                 ctypes.byref(o), _lib.SPE_STAGE_DECODE), "spe_forward_stages")
        return out

    def forward(self, samples, clip_bbox=None, stream=None, return_hs=False):
        """REV/models/detr_speed.py:59-92.  Returns pred_logits [B,Q,12], pred_points [B,Q,2]
        (+ pred_sigmas as log-sigma when the sigma head is configured).  Passing `clip_bbox`
        ([B,4] device fp32) also runs the fused PostProcess and adds `probs` / `points_px`."""
        if self._handle is None:
            raise RuntimeError("DETR: load_state_dict() with every parameter before forward()")
        if isinstance(samples, (list, tuple)):            # REV/models/detr_speed.py:74-75
            samples = nested_tensor_from_tensor_list(list(samples))
        images = samples.tensors if isinstance(samples, NestedTensor) else samples
        if not images.is_cuda:
            raise RuntimeError("DETR (HIP) expects device tensors; call samples.to('cuda')")
        if images.dtype == torch.uint8:
            # the 8-bit crops to_tensor + Normalize would make the batch from (spe_forward_stages_u8)
            ch = self._crop_channels(images)
            B, dev = images.shape[0], images.device
            if clip_bbox is not None:
                clip_bbox = clip_bbox.to(device=dev, dtype=torch.float32).contiguous()
            out, o = self._outputs(B, dev, clip_bbox, return_hs)
            ws = self.workspace(B, dev, stream)
            _lib.check(_lib.lib().spe_forward_stages_u8(self._h, _lib.stream_ptr(stream), _lib.ptr(images), ch, B,
                                                        _lib.ptr(ws), ws.numel(), ctypes.byref(o),
                                                        _lib.SPE_STAGE_ENCODE | _lib.SPE_STAGE_DECODE),
                       "spe_forward_stages_u8")
            return out
        images = images.contiguous().float()
        B, C, H, W = images.shape
        S = self.cfg.input_size
        if C != 3 or H != S or W != S:
            raise ValueError(f"expected [B,3,{S},{S}] input, got {tuple(images.shape)}")
        dev = images.device
        if clip_bbox is not None:
            clip_bbox = clip_bbox.to(device=dev, dtype=torch.float32).contiguous()
        out, o = self._outputs(B, dev, clip_bbox, return_hs)
        ws = self.workspace(B, dev, stream)
        _lib.check(_lib.lib().spe_forward(self._h, _lib.stream_ptr(stream), _lib.ptr(images), B, _lib.ptr(ws),
                                          ws.numel(), ctypes.byref(o)), "spe_forward")
        return out

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                _lib.lib().spe_model_destroy(self._h)
                self._h = None
        except Exception:
            pass


class SetCriterion(nn.Module):
    """REV/models/detr_speed.py:103-261 with the HungarianMatcher of REV/models/matcher.py:35-88,
    on the device (spe_criterion, csrc/criterion.hip): one launch matches and scores the last
    layer and every aux layer.  Returns the reference's loss dict (loss_ce, class_error,
    loss_points, cardinality_error, and *_i for aux layer i without class_error) as 0-d device
    tensors; `weight_dict` as REV/models/detr_speed.py:319-327 builds it.  The matching of the
    last call is kept in `last_match` ([L,B,T] query per target; layer L-1 = last)."""

    def __init__(self, num_classes: int = 11, cost_class: float = 1.0, cost_pts: float = 5.0,
                 eos_coef: float = 0.1, pts_loss_coef: float = 5.0, dec_layers: int = 6, aux_loss: bool = True):
        super().__init__()
        self.num_classes, self.cost_class, self.cost_pts, self.eos_coef = num_classes, cost_class, cost_pts, eos_coef
        self.weight_dict = {"loss_ce": 1, "loss_points": pts_loss_coef}
        if aux_loss:
            for i in range(dec_layers - 1):
                self.weight_dict.update({f"loss_ce_{i}": 1, f"loss_points_{i}": pts_loss_coef})
        self.last_match = None

    @torch.no_grad()
    def forward(self, outputs, targets, stream=None):
        layers = [(a["pred_logits"], a["pred_points"]) for a in outputs.get("aux_outputs", [])]
        layers.append((outputs["pred_logits"], outputs["pred_points"]))
        logits = torch.stack([l for l, _ in layers]).float().contiguous()
        points = torch.stack([p for _, p in layers]).float().contiguous()
        L, B, Q, C = logits.shape
        dev = logits.device
        labels = torch.stack([t["labels"] for t in targets]).to(dev, torch.int32).contiguous()
        tpts = torch.stack([t["landmarks"] for t in targets]).to(dev, torch.float32).contiguous()
        T = labels.shape[1]
        num_points = float(B * T)                         # REV/models/detr_speed.py:235-244
        from . import dist as spe_dist
        if spe_dist.is_dist():
            n = torch.tensor([num_points], dtype=torch.float64, device=dev)
            torch.distributed.all_reduce(n)
            num_points = float(n.item()) / torch.distributed.get_world_size()
        num_points = max(num_points, 1.0)
        match = torch.empty(L, B, T, dtype=torch.int32, device=dev)
        res = torch.empty(L, 4, dtype=torch.float64, device=dev)
        _lib.check(_lib.lib().spe_criterion(_lib.stream_ptr(stream), _lib.ptr(logits), _lib.ptr(points), _lib.ptr(labels),
                                            _lib.ptr(tpts), L, B, Q, C, T, self.cost_class, self.cost_pts,
                                            self.eos_coef, num_points, _lib.ptr(match), _lib.ptr(res)), "spe_criterion")
        self.last_match = match
        losses = {}
        for l in range(L):
            sfx = "" if l == L - 1 else f"_{l}"
            losses["loss_ce" + sfx] = res[l, 0]
            if l == L - 1:
                losses["class_error"] = res[l, 1]
            losses["cardinality_error" + sfx] = res[l, 2]
            losses["loss_points" + sfx] = res[l, 3]
        return losses


class PostProcess(nn.Module):
    """REV/models/detr_speed.py:264-293 (and the sigma variant,
    UNC/src/zoo/rtdetr/rtdetr_postprocessor.py:44-78): softmax over the 12 classes and
    crop -> image pixel rescale, on device; returns the reference's list of numpy dicts."""

    @torch.no_grad()
    def forward(self, outputs, clip_bbox, stream=None):
        logits, points = outputs["pred_logits"], outputs["pred_points"]
        B, Q, _ = logits.shape
        assert len(clip_bbox) == B
        dev = logits.device
        bb = torch.stack([torch.as_tensor(b, dtype=torch.float32) for b in clip_bbox]).to(dev)
        if "probs" in outputs and "points_px" in outputs:
            probs, pts = outputs["probs"], outputs["points_px"]
        else:
            probs = torch.empty_like(logits)
            pts = torch.empty_like(points)
            _lib.check(_lib.lib().spe_postprocess(_lib.stream_ptr(stream), _lib.ptr(logits.contiguous()),
                                                   _lib.ptr(points.contiguous()), _lib.ptr(bb), B, Q,
                                                   _lib.ptr(probs), _lib.ptr(pts)), "spe_postprocess")
        probs, pts = probs.cpu().numpy(), pts.cpu().numpy()
        res = [{"logits": probs[i], "points": pts[i]} for i in range(B)]
        if "sigmas" in outputs:
            sg = outputs["sigmas"].cpu().numpy()
            for i in range(B):
                res[i]["sigmas"] = sg[i]
        return res


def build_model(args, dtype: str = None):
    """REV/models/__init__.py:5-6 / detr_speed.py:296-336.  Returns (model, criterion,
    postprocessors); the criterion is the device SetCriterion with the reference's argparse
    defaults (set_cost_class 1, set_cost_pts 5, eos_coef 0.1, pts_loss_coef 5)."""
    cfg = SpeConfig.from_args(args)
    dtype = dtype or getattr(args, "dtype", "bf16")
    aux = bool(getattr(args, "aux_loss", False))
    model = DETR(cfg, dtype=dtype, aux_loss=aux, attn_dtype=getattr(args, "attn_dtype", None))
    criterion = SetCriterion(cost_class=float(getattr(args, "set_cost_class", 1.0)),
                             cost_pts=float(getattr(args, "set_cost_pts", 5.0)),
                             eos_coef=float(getattr(args, "eos_coef", 0.1)),
                             pts_loss_coef=float(getattr(args, "pts_loss_coef", 5.0)),
                             dec_layers=cfg.dec_layers, aux_loss=aux)
    return model, criterion, {"points": PostProcess()}
