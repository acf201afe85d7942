"""Full-size BASELINE configurations on the HIP path (c2 lives in
test_parity_gpu.py): c3 (10M observations, RPC d=2), its RPC d=3 variant with
Jacobian planes past 2^31 elements, c4 (50M observations as its 8 landmark
shards, the per-GPU problems of the 8-GPU run) and c5 (1M reprojection + ~250k
depth blocks).

Per configuration, on the device planes (mvba_evaluate_device):
  * determinism: two residual+Jacobian evaluations are bit-identical;
  * residual-only equals residual+Jacobian residuals, bit for bit;
  * the device order is a permutation of the residual blocks;
  * a seeded random sample of residual blocks against the oracle's exact
    derivative (oracle.ANALYTIC, rig_calibrator.cc:447-482 + rpc_distortion.cc:116-160):
    residuals <= 1e-9 x max(|pixel|, 1), every written Jacobian entry <= 1e-9 of
    its column maximum;
  * c5: a sample of depth blocks against oracle_depth_error (rig_calibrator.cc:547-583)
    at the same tolerances.
"""
import multiprocessing as mp
from concurrent.futures import ProcessPoolExecutor

import numpy as np
import pytest

from multiview_amd import _lib, rig
from multiview_amd.evaluator import Evaluator

pytestmark = pytest.mark.gpu

INT32_LIMIT = 2 ** 31


def _check_sample(P, oracle, r_g, J_g, idx):
    sub = P.subset(idx)
    _, r_o, J_o = oracle.evaluate(sub, oracle.ANALYTIC)
    pix = np.maximum(np.abs(sub.residual_meas + r_o).max(axis=1), 1.0)
    assert np.all(np.abs(r_g - r_o) <= 1e-9 * pix[:, None]), np.abs(r_g - r_o).max()
    colmax = np.maximum(np.abs(J_o).max(axis=0), 1e-12)
    written = J_o != 0
    err = np.abs(J_g - J_o)[written] / np.broadcast_to(colmax, J_o.shape)[written]
    assert err.max() <= 1e-9, err.max()
    return r_o, J_o


def _full_size_properties(P, oracle, sample, seed, ld=None):
    """Determinism, residual-only agreement, permutation and a random oracle
    sample on one problem. The Jacobian planes start NaN-filled (entries of
    constant blocks are never written, as Ceres passes NULL for them). Returns
    a summary dict (sizes, last valid slot and its column) for further checks."""
    import torch

    out = {}
    with Evaluator(P) as ev:
        ev.set_params()
        n, S = ev.num_residuals, ev.num_slots
        ld = ld or ev.ld
        j1 = torch.full((ev.stride, ld), float("nan"), dtype=torch.float64, device="cuda")
        r1 = torch.empty((2, ld), dtype=torch.float64, device="cuda")
        ev.evaluate_device(True, residuals=r1, jac=j1, ld=ld)
        ev.sync()
        order = ev.order()
        valid_np = order >= 0
        assert np.array_equal(np.sort(order[valid_np]), np.arange(n))
        valid = torch.from_numpy(valid_np).cuda()
        # residual-only pass into a second buffer
        r3 = torch.empty_like(r1)
        ev.evaluate_device(False, residuals=r3, jac=None, ld=ld)
        ev.sync()
        assert torch.equal(r1[:, :S][:, valid], r3[:, :S][:, valid])
        del r3
        # random sample against the oracle
        rng = np.random.default_rng(seed)
        slots = np.nonzero(valid_np)[0]
        pos = np.sort(rng.choice(slots, sample, replace=False))
        pos_t = torch.from_numpy(pos).cuda()
        r_g = r1[:, pos_t].T.cpu().numpy()
        J_g = j1[:, pos_t].T.cpu().numpy()
        _check_sample(P, oracle, r_g, J_g, order[pos])
        # determinism: a second residual+Jacobian evaluation, bit-identical
        # (compared plane by plane so only one extra plane set is resident)
        j2 = torch.full_like(j1, float("nan"))
        r2 = torch.empty_like(r1)
        ev.evaluate_device(True, residuals=r2, jac=j2, ld=ld)
        ev.sync()
        assert torch.equal(r1[:, :S][:, valid], r2[:, :S][:, valid])
        eq = (j1[:, :S] == j2[:, :S]) | (torch.isnan(j1[:, :S]) & torch.isnan(j2[:, :S]))
        assert bool(eq[:, valid].all())
        del j2, r2, eq
        last = int(slots[-1])
        out.update(n=n, S=S, ld=ld, stride=ev.stride, last_slot=last, last_index=int(order[last]),
                   last_col=j1[:, last].cpu().numpy(), last_res=r1[:, last].cpu().numpy())
        del j1, r1
        torch.cuda.empty_cache()
    return out


def test_full_size_c3(oracle):
    """c3: 3-sensor rig, 1M landmarks, ~10M observations, RPC degree 2 (K = 44)."""
    R = rig.make_rig(**rig.CONFIGS["c3"])
    P = rig.build_problem(R)
    assert P.num_residuals > 9_500_000
    _full_size_properties(P, oracle, sample=4000, seed=31)


def test_full_size_c3_rpc3_planes_past_int32(oracle):
    """c3's RPC d=3 variant (K = 76, 208 Jacobian planes): with a leading
    dimension that puts the last planes beyond 2^31 elements the int64 plane
    indexing (mvba_kernels.hip, stj) is exercised. The planes start NaN-filled;
    at the last valid slot every entry of the last plane set is checked: the
    RPC undistortion half (last plane) is exactly 0 (written, not skipped:
    Ceres' numeric Jacobian of an unused coefficient), the distortion half and
    the residual against the oracle."""
    cfg = dict(rig.CONFIGS["c3"], models=["rpc3"] * 3)
    R = rig.make_rig(**cfg)
    P = rig.build_problem(R)
    K = 76
    stride = 56 + 2 * K
    ld = ((INT32_LIMIT // (stride - 1) + 4096 + 63) // 64) * 64
    assert (stride - 1) * ld > INT32_LIMIT  # the whole last plane lies past 2^31 elements
    info = _full_size_properties(P, oracle, sample=3000, seed=37, ld=ld)
    assert info["stride"] == stride and info["ld"] == ld
    col, res = info["last_col"], info["last_res"]
    assert col[stride - 1] == 0.0  # undistortion half, last coefficient, row y
    assert np.all(col[_lib.JAC_BASE[7] + K // 2:_lib.JAC_BASE[7] + K] == 0.0)  # row x undistortion half
    assert np.all(col[_lib.JAC_BASE[7] + K + K // 2:] == 0.0)
    r_o, J_o = _check_sample(P, oracle, res[None, :], col[None, :], np.array([info["last_index"]]))
    dist_rows = np.r_[_lib.JAC_BASE[7]:_lib.JAC_BASE[7] + K // 2, _lib.JAC_BASE[7] + K:_lib.JAC_BASE[7] + K + K // 2]
    assert np.all(np.isfinite(col[dist_rows]))
    assert np.abs(J_o[0, dist_rows]).max() > 0.0


def _c4_shard(rank):
    cfg = dict(rig.CONFIGS["c4"])
    npts, world = cfg["num_points"], 8
    cfg["point_range"] = (rank * npts // world, (rank + 1) * npts // world)
    return rig.build_problem(rig.make_rig(**cfg))


def test_full_size_c4_shards(oracle):
    """c4: 8-sensor rig, 5M landmarks, 50M observations, as 8 landmark-range
    shards (make_rig point ranges: each shard's landmarks from its own stream;
    bench.py cuts the whole problem in capture order instead, rig.shard_points),
    each evaluated on this GPU.
    Shards are generated by 8 worker processes (CPU only) while the GPU checks
    the previous ones."""
    total = 0
    ctx = mp.get_context("fork")
    with ProcessPoolExecutor(max_workers=8, mp_context=ctx) as pool:
        for rank, P in enumerate(pool.map(_c4_shard, range(8))):
            total += P.num_residuals
            _full_size_properties(P, oracle, sample=500, seed=100 + rank)
            del P
    assert total > 45_000_000


def test_full_size_c5_reprojection_and_depth(oracle):
    """c5: 3 image + 1 image+depth sensors, ~1M reprojection and ~250k depth
    blocks (depth_tri_weight 10, depth_to_image and scale floating)."""
    import torch

    R = rig.make_rig(**rig.CONFIGS["c5"])
    P = rig.build_problem(R, rig.FloatFlags(**rig.CONFIG_FLAGS["c5"]))
    assert P.num_depth_residuals > 200_000
    _full_size_properties(P, oracle, sample=4000, seed=41)
    with Evaluator(P) as ev:
        ev.set_params()
        nd, S = ev.num_depth, ev.num_depth_slots
        dld = (S + 63) // 64 * 64
        planes = []
        for jac in (True, True, False):
            r = torch.empty((3, dld), dtype=torch.float64, device="cuda")
            J = torch.full((_lib.DJAC_ROWS, dld), float("nan"), dtype=torch.float64, device="cuda") if jac else None
            ev.evaluate_depth_device(jac, residuals=r, jac=J, ld=dld)
            planes.append((r, J))
        ev.sync()
        order = ev.depth_order()
        valid_np = order >= 0
        assert np.array_equal(np.sort(order[valid_np]), np.arange(nd))
        valid = torch.from_numpy(valid_np).cuda()
        (r1, J1), (r2, J2), (r3, _) = planes
        assert torch.equal(r1[:, :S][:, valid], r2[:, :S][:, valid])
        assert torch.equal(r1[:, :S][:, valid], r3[:, :S][:, valid])
        eq = (J1[:, :S] == J2[:, :S]) | (torch.isnan(J1[:, :S]) & torch.isnan(J2[:, :S]))
        assert bool(eq[:, valid].all())
        rng = np.random.default_rng(43)
        pos = np.sort(rng.choice(np.nonzero(valid_np)[0], 1500, replace=False))
        pos_t = torch.from_numpy(pos).cuda()
        r_g = r1[:, pos_t].T.cpu().numpy()
        J_g = J1[:, pos_t].T.cpu().numpy()
    idx = order[pos]
    sub = rig.build_problem(R, rig.FloatFlags(**rig.CONFIG_FLAGS["c5"]))
    sub.depth_blocks = P.depth_blocks[idx]
    sub.depth_meas = P.depth_meas[idx]
    sub.depth_weight = P.depth_weight[idx]
    sub.depth_stamps = P.depth_stamps[idx]
    sub.depth_after = P.depth_after[idx]
    _, r_o, J_o = oracle.evaluate_depth(sub, oracle.ANALYTIC)
    assert np.abs(r_g - r_o).max() <= 1e-9 * max(np.abs(r_o).max(), 1.0)
    for b in range(7):
        lo, hi = _lib.DJAC_BASE[b], (_lib.DJAC_BASE[b + 1] if b < 6 else _lib.DJAC_ROWS)
        ref = J_o[:, lo:hi]
        written = ref != 0
        if not written.any():
            continue
        scale = np.abs(ref).max()
        assert np.abs(J_g[:, lo:hi] - ref)[written].max() <= 1e-9 * scale, b
