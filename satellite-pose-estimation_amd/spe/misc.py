"""Batching helpers with the reference's contract (REV/utils/misc.py:272-333)."""
from __future__ import annotations

from typing import List, Optional

import torch
from torch import Tensor


class NestedTensor:
    """Images [B,3,H,W] + padding mask [B,H,W] (True on padding), REV/utils/misc.py:287-308."""

    def __init__(self, tensors: Tensor, mask: Optional[Tensor]):
        self.tensors = tensors
        self.mask = mask

    def to(self, device, non_blocking=False):
        m = self.mask.to(device, non_blocking=non_blocking) if self.mask is not None else None
        return NestedTensor(self.tensors.to(device, non_blocking=non_blocking), m)

    def decompose(self):
        return self.tensors, self.mask

    def __repr__(self):
        return repr(self.tensors)


def nested_tensor_from_tensor_list(tensor_list: List[Tensor]) -> NestedTensor:
    """Zero-pad to the largest image, mask True on padding (REV/utils/misc.py:311-333).
    The HIP path serves fixed-size crops (mask all False), which is what the reference's
    SPEED loaders produce; padded batches are rejected by DETR.forward's shape check."""
    if tensor_list[0].ndim != 3:
        raise ValueError("not supported")
    c = max(t.shape[0] for t in tensor_list)
    h = max(t.shape[1] for t in tensor_list)
    w = max(t.shape[2] for t in tensor_list)
    b = len(tensor_list)
    dev, dt = tensor_list[0].device, tensor_list[0].dtype
    tensor = torch.zeros((b, c, h, w), dtype=dt, device=dev)
    mask = torch.ones((b, h, w), dtype=torch.bool, device=dev)
    for img, pad, m in zip(tensor_list, tensor, mask):
        pad[: img.shape[0], : img.shape[1], : img.shape[2]].copy_(img)
        m[: img.shape[1], : img.shape[2]] = False
    return NestedTensor(tensor, mask)


def collate_fn(batch):
    """REV/utils/misc.py:272-275."""
    batch = list(zip(*batch))
    batch[0] = nested_tensor_from_tensor_list(batch[0])
    return tuple(batch)
