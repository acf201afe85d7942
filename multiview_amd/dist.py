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
    """libamdhip64 (already loaded by torch) for raw-pointer copies in the host
    callback path."""
    global _HIP
    if _HIP is None:
        import ctypes as C

        lib = C.CDLL("libamdhip64.so")
        lib.hipMemcpy.restype = C.c_int
        lib.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        lib.hipStreamSynchronize.restype = C.c_int
        lib.hipStreamSynchronize.argtypes = [C.c_void_p]
        _HIP = lib
    return _HIP


class _DevicePtr:
    """A library-owned device buffer seen by torch without a copy."""

    def __init__(self, ptr: int, count: int):
        self.__cuda_array_interface__ = {"shape": (count,), "typestr": "<f8", "data": (ptr, False),
                                         "version": 2, "strides": None}


class SolverExchange:
    """The mvba_allreduce_fn of a sharded mvba_solve over torch.distributed.

    Stream-ordered (the ABI contract, include/mvba/mvba.h): with the RCCL
    backend ("nccl") the library's device buffer is wrapped as a tensor (no
    copy) and all-reduced in place on the solver's stream — no host wait. With
    gloo (CPU rehearsal) the callback synchronises the stream, stages the
    buffer through host memory and copies the result back before returning."""

    H2D, D2H = 1, 2

    def __init__(self, device=None):
        import torch
        import torch.distributed as dist

        self.dist = dist
        self.on_device = dist.get_backend() == "nccl"
        self.device = device
        self.host = torch.empty(0, dtype=torch.float64)
        self.views = {}
        self.calls = 0
        self.doubles = 0

    def _view(self, ptr, count):
        import torch

        key = (ptr, count)
        v = self.views.get(key)
        if v is None:
            v = torch.as_tensor(_DevicePtr(ptr, count), device=torch.device("cuda", self.device or 0))
            self.views[key] = v
        return v

    def __call__(self, ptr: int, count: int, op: int, stream: int = 0):
        import torch

        red = self.dist.ReduceOp.SUM if op == 0 else self.dist.ReduceOp.MAX
        if self.on_device:
            st = torch.cuda.ExternalStream(stream) if stream else torch.cuda.default_stream()
            with torch.cuda.stream(st):
                self.dist.all_reduce(self._view(ptr, count), op=red)
        else:
            hip = _hip()
            if hip.hipStreamSynchronize(stream or None) != 0:
                raise RuntimeError("hipStreamSynchronize failed")
            if self.host.numel() < count:
                self.host = torch.empty(max(count, 2 * self.host.numel()), dtype=torch.float64)
            view = self.host[:count]
            if hip.hipMemcpy(view.data_ptr(), ptr, count * 8, self.D2H) != 0:
                raise RuntimeError("hipMemcpy into the exchange buffer failed")
            self.dist.all_reduce(view, op=red)
            if hip.hipMemcpy(ptr, view.data_ptr(), count * 8, self.H2D) != 0:
                raise RuntimeError("hipMemcpy out of the exchange buffer failed")
        self.calls += 1
        self.doubles += count


class Comm:
    """A library-native communicator (mvba_comm, include/mvba/mvba.h) for the
    solver option ``comm=``: the exchange is ``mvba_comm_allreduce``, enqueued
    on the solver's stream in C++ (no Python in the CG loop).

    Comm.rccl(device): one process per GPU over torch.distributed — rank 0's
    RCCL unique id is broadcast with torch.distributed, then every rank joins.
    Comm.local(devices): several shards in one process (one thread and stream
    per shard), returns one Comm per shard."""

    def __init__(self, handle):
        from . import _lib

        self.lib = _lib.load()
        self.h = handle

    @classmethod
    def rccl(cls, device: int, timeout_s: float = 0.0):
        """timeout_s: deadline of the communicator's init and of every
        collective enqueue (<= 0: MVBA_COMM_TIMEOUT_S, else 300 s); past it the
        communicator is aborted and the call raises instead of hanging."""
        import ctypes as C

        import numpy as np
        import torch
        import torch.distributed as dist

        from . import _lib

        lib = _lib.load()
        ident = np.zeros(_lib.COMM_ID_BYTES, dtype=np.uint8)
        if dist.get_rank() == 0:
            _lib.check(lib.mvba_comm_unique_id(ident.ctypes.data))
        t = torch.from_numpy(ident)
        if dist.get_backend() == "nccl":
            t = t.cuda(device)
        dist.broadcast(t, 0)
        ident = np.ascontiguousarray(t.cpu().numpy())
        h = C.c_void_p()
        st = lib.mvba_comm_init_rccl_deadline(ident.ctypes.data, dist.get_world_size(), dist.get_rank(), device,
                                              float(timeout_s), C.byref(h))
        if st != 0:
            raise _lib.MvbaError(st, lib.mvba_comm_error().decode())
        return cls(h)

    @classmethod
    def rccl_world1(cls, device: int, timeout_s: float = 0.0):
        """A one-rank RCCL communicator without torch.distributed (the unique
        id stays in this process): the exchange path of a sharded solve
        (ncclAllReduce on the solver's stream, the fold-mode CG tail, captured
        CG runs) rehearsed on one GPU; the all-reduce is an identity there."""
        import ctypes as C

        import numpy as np

        from . import _lib

        lib = _lib.load()
        ident = np.zeros(_lib.COMM_ID_BYTES, dtype=np.uint8)
        _lib.check(lib.mvba_comm_unique_id(ident.ctypes.data))
        h = C.c_void_p()
        st = lib.mvba_comm_init_rccl_deadline(ident.ctypes.data, 1, 0, device, float(timeout_s), C.byref(h))
        if st != 0:
            raise _lib.MvbaError(st, lib.mvba_comm_error().decode())
        return cls(h)

    @classmethod
    def local(cls, devices):
        import ctypes as C

        import numpy as np

        from . import _lib

        lib = _lib.load()
        dev = np.ascontiguousarray(devices, dtype=np.int32)
        out = (C.c_void_p * len(dev))()
        st = lib.mvba_comm_init_local(len(dev), dev.ctypes.data, out)
        if st != 0:
            raise _lib.MvbaError(st, lib.mvba_comm_error().decode())
        return [cls(C.c_void_p(out[i])) for i in range(len(dev))]

    def allreduce(self, ptr: int, count: int, op: int = 0, stream: int = 0):
        """mvba_comm_allreduce on a device buffer, enqueued on `stream` (the
        solver's exchange, callable on its own for timing)."""
        import ctypes as C

        if self.lib.mvba_comm_allreduce(C.c_void_p(ptr), count, op, C.c_void_p(stream), self.h) != 0:
            raise RuntimeError("mvba_comm_allreduce failed: " + self.lib.mvba_comm_error().decode())

    def abort(self):
        if self.h is not None and self.h.value:
            self.lib.mvba_comm_abort(self.h)

    def close(self):
        if self.h is not None and self.h.value:
            self.lib.mvba_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
