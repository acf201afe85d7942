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


_HIP = None


def _hip():
    """libamdhip64 (already loaded by torch) for raw-pointer copies in the callback."""
    global _HIP
    if _HIP is None:
        import ctypes as C

        lib = C.CDLL("libamdhip64.so")
        lib.hipMemcpy.restype = C.c_int
        lib.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        _HIP = lib
    return _HIP


class SolverExchange:
    """The mvba_allreduce_fn of a sharded mvba_solve, over torch.distributed.

    The library hands a raw device pointer; it is staged through a persistent
    buffer (device memory for RCCL — backend "nccl" — host memory for gloo),
    all-reduced in place, and copied back. Calls are synchronous, as the ABI
    requires."""

    H2D, D2H, D2D = 1, 2, 3

    def __init__(self, device=None):
        import torch
        import torch.distributed as dist

        self.dist = dist
        self.on_device = dist.get_backend() == "nccl"
        self.device = device if self.on_device else "cpu"
        self.buf = torch.empty(0, dtype=torch.float64, device=self.device)
        self.calls = 0
        self.doubles = 0

    def __call__(self, ptr: int, count: int, op: int):
        import torch

        if self.buf.numel() < count:
            self.buf = torch.empty(max(count, 2 * self.buf.numel()), dtype=torch.float64, device=self.device)
        view = self.buf[:count]
        nbytes = count * 8
        kind_in = self.D2D if self.on_device else self.D2H
        kind_out = self.D2D if self.on_device else self.H2D
        hip = _hip()
        if self.on_device:
            torch.cuda.synchronize(self.device)
        if hip.hipMemcpy(view.data_ptr(), ptr, nbytes, kind_in) != 0:
            raise RuntimeError("hipMemcpy into the exchange buffer failed")
        self.dist.all_reduce(view, op=self.dist.ReduceOp.SUM if op == 0 else self.dist.ReduceOp.MAX)
        if self.on_device:
            torch.cuda.synchronize(self.device)
        if hip.hipMemcpy(ptr, view.data_ptr(), nbytes, kind_out) != 0:
            raise RuntimeError("hipMemcpy out of the exchange buffer failed")
        self.calls += 1
        self.doubles += count
