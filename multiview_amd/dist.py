"""Landmark-range sharding and the per-iteration exchange.

Observations shard by landmark range: rank r owns landmarks [lo_r, hi_r) and
all their observations; every rank holds all camera-side parameters. The
normal equations then split into
  * point blocks (V_p, g_p): rank-local, never exchanged;
  * camera-side gradient + block-diagonal Hessian: partial sums on every rank,
    summed with ONE all-reduce per iteration (RCCL over xGMI on MI355X, gloo on
    CPU for tests), payload = cam_grad_size + cam_hess_size + 1 (cost) doubles.
"""
from __future__ import annotations

import hashlib

import numpy as np


def shard_range(num_points: int, world: int, rank: int):
    """Contiguous landmark range of a rank (equal split, remainder to the first ranks)."""
    base, extra = divmod(num_points, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def layout_fingerprint(layout: dict, block_sizes: np.ndarray) -> int:
    """Hash of the camera-side layout (block sizes in order + offsets): must be equal
    on every rank for the all-reduce to be meaningful."""
    sizes = np.asarray(block_sizes)[layout["cam_block_ids"]].astype(np.int64)
    h = hashlib.sha256()
    h.update(sizes.tobytes())
    h.update(np.asarray(layout["cam_goff"], dtype=np.int64).tobytes())
    h.update(np.asarray(layout["cam_hoff"], dtype=np.int64).tobytes())
    return int.from_bytes(h.digest()[:7], "little")


def check_layouts_agree(layout: dict, block_sizes: np.ndarray, device=None):
    import torch
    import torch.distributed as dist

    fp = torch.tensor([layout_fingerprint(layout, block_sizes)], dtype=torch.int64, device=device)
    lo, hi = fp.clone(), fp.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    if lo.item() != hi.item():
        raise RuntimeError("camera-side normal-equation layouts differ across ranks")


class NormalEquationBuffer:
    """One flat buffer [cam_grad | cam_hess | cost] so the exchange is a single
    all-reduce; views are handed to mvba_linearize_device."""

    def __init__(self, layout: dict, device, dtype=None):
        import torch

        self.ng = int(layout["cam_grad_size"])
        self.nh = int(layout["cam_hess_size"])
        self.flat = torch.zeros(self.ng + self.nh + 1, dtype=dtype or torch.float64, device=device)
        self.grad = self.flat[: self.ng]
        self.hess = self.flat[self.ng: self.ng + self.nh]
        self.cost = self.flat[self.ng + self.nh:]

    @property
    def payload_bytes(self) -> int:
        return self.flat.numel() * self.flat.element_size()

    def allreduce(self):
        import torch.distributed as dist

        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM)
