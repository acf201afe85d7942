"""World-size-2 gloo test of the landmark-range sharding and the camera-side
normal-equation all-reduce, on CPU.

Each rank builds its shard (points [lo, hi) of a global rig), linearizes it with
the oracle's exact Jacobian (the reference for the GPU kernels), all-reduces the
camera-side buffer with multiview_amd.dist, and compares with the unsharded
problem. The GPU path runs the same helper with RCCL (bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Layout:
    """Camera-side layout computed on the host exactly as mvba_create does:
    non-constant, non-point blocks in block-id order."""

    @staticmethod
    def of(P):
        is_pt = np.zeros(len(P.block_size), dtype=bool)
        is_pt[np.unique(P.residual_blocks[:, 3])] = True
        ids = np.nonzero(~is_pt & (P.block_constant == 0))[0].astype(np.int32)
        sz = P.block_size[ids].astype(np.int64)
        goff = np.concatenate([[0], np.cumsum(sz)[:-1]]) if len(sz) else np.zeros(0, np.int64)
        hoff = np.concatenate([[0], np.cumsum(sz * sz)[:-1]]) if len(sz) else np.zeros(0, np.int64)
        pts = np.unique(P.residual_blocks[:, 3])
        # point index order = first appearance in residual order
        _, first = np.unique(P.residual_blocks[:, 3], return_index=True)
        pts = P.residual_blocks[np.sort(first), 3].astype(np.int32)
        return dict(cam_grad_size=int(sz.sum()), cam_hess_size=int((sz * sz).sum()),
                    num_points=len(pts), cam_block_ids=ids, cam_goff=goff.astype(np.int64),
                    cam_hoff=hoff.astype(np.int64), point_block_ids=pts, supported=True)


CFG = dict(num_sensors=3, num_ref=12, num_points=400, obs_per_point=5, models=["radtan", "fov", "rpc1"], seed=21)


def _linearize(P):
    from oracle.normal_equations import normal_equations_reference
    from oracle import oracle_py

    L = _Layout.of(P)
    c, r, J = oracle_py.evaluate(P, oracle_py.ANALYTIC, apply_loss=True, robust_threshold=3.0)
    g, h, _, _ = normal_equations_reference(P, r, J, L)
    return L, g, h, c


def _worker(rank, world, port, out_dir):
    import sys

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist

    from multiview_amd import rig
    from multiview_amd.dist import NormalEquationBuffer, check_layouts_agree, shard_range

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(CFG["num_points"], world, rank)
    R = rig.make_rig(**dict(CFG, point_range=(lo, hi)))
    P = rig.build_problem(R)
    L, g, h, c = _linearize(P)
    check_layouts_agree(L, P.block_size)
    buf = NormalEquationBuffer(L, device="cpu")
    buf.grad.copy_(torch.from_numpy(g))
    buf.hess.copy_(torch.from_numpy(h))
    buf.cost.fill_(c)
    buf.allreduce()
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), buf.flat.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_normal_equations_allreduce(tmp_path):
    world = 2
    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    flats = [np.load(tmp_path / f"rank{r}.npy") for r in range(world)]
    assert np.array_equal(flats[0], flats[1])
    # unsharded reference: the union of the shards' landmarks
    from multiview_amd import rig

    parts = []
    for r in range(world):
        from multiview_amd.dist import shard_range

        lo, hi = shard_range(CFG["num_points"], world, r)
        parts.append(rig.make_rig(**dict(CFG, point_range=(lo, hi))))
    # combine shards into one problem: same cameras, concatenated points/observations
    R0 = parts[0]
    off = 0
    xyz, init_xyz, pid, cid, pix = [], [], [], [], []
    for Rk in parts:
        xyz.append(Rk.xyz)
        init_xyz.append(Rk.init["xyz"])
        pid.append(Rk.obs_pid + off)
        cid.append(Rk.obs_cid)
        pix.append(Rk.obs_pix)
        off += Rk.xyz.shape[0]
    R0.xyz = np.concatenate(xyz)
    R0.init["xyz"] = np.concatenate(init_xyz)
    R0.obs_pid, R0.obs_cid, R0.obs_pix = np.concatenate(pid), np.concatenate(cid), np.concatenate(pix)
    P = rig.build_problem(R0)
    L, g, h, c = _linearize(P)
    ng, nh = L["cam_grad_size"], L["cam_hess_size"]
    assert flats[0].size == ng + nh + 1
    scale_g = np.abs(g).max()
    scale_h = np.abs(h).max()
    assert np.abs(flats[0][:ng] - g).max() <= 1e-10 * scale_g
    assert np.abs(flats[0][ng:ng + nh] - h).max() <= 1e-10 * scale_h
    assert np.isclose(flats[0][-1], c, rtol=1e-12)


def test_shard_range_partitions():
    from multiview_amd.dist import shard_range

    for n, w in [(10, 3), (100000, 8), (7, 8)]:
        rs = [shard_range(n, w, r) for r in range(w)]
        assert rs[0][0] == 0 and rs[-1][1] == n
        assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
