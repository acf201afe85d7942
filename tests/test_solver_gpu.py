"""GPU Levenberg-Marquardt (mvba_solve) against the CPU reference LM
(oracle/lm_reference.py: Ceres 1.14 control flow, exact dense linear solves).

* one LM iteration with CG run to convergence (eta ~ 0) must equal the exact
  step: relative 1e-8;
* full solves (Ceres tolerances of rig_calibrator.cc:1914-1917) must converge to
  the same parameters: |dx| <= 1e-6 max(1, |x|) (north_star), cost rtol 1e-9;
* a landmark-sharded solve over two ranks (gloo exchange through the
  mvba_allreduce_fn callback, both ranks on cuda:0) must match the unsharded one.
Problems keep the reference poses constant (camera_poses_to_float empty) so the
minimum is unique (no gauge freedom)."""
import os
import socket

import numpy as np
import pytest

from conftest import ROOT
from multiview_amd import rig
from multiview_amd.evaluator import Evaluator

pytestmark = pytest.mark.gpu

TOL = dict(function_tolerance=1e-16, gradient_tolerance=1e-16, parameter_tolerance=1e-12)
FLAGS = rig.FloatFlags(camera_poses_to_float=())


def _problem(models, seed, num_points=300, flags=FLAGS):
    R = rig.make_rig(num_sensors=len(models), num_ref=12, num_points=num_points, obs_per_point=5,
                     models=models, seed=seed)
    P = rig.build_problem(R, flags)
    return R, P


def _close(a, b, rel):
    return np.abs(a - b).max() <= rel * max(1.0, np.abs(b).max())


def _free_mask(P):
    m = np.zeros(P.params.size, dtype=bool)
    for b in np.nonzero(P.block_constant == 0)[0]:
        o = int(P.block_offset[b])
        m[o:o + int(P.block_size[b])] = True
    return m


@pytest.mark.parametrize("use_loss", [False, True])
def test_one_exact_step_matches_dense_lm(use_loss):
    from oracle import lm_reference

    _, P = _problem(["radtan", "fov", "rpc1"], seed=31)
    x_ref, s_ref = lm_reference.solve(P, max_num_iterations=1, use_loss=use_loss, **TOL)
    with Evaluator(P) as ev:
        ev.set_params()
        s = ev.solve(max_num_iterations=1, eta=1e-14, max_linear_solver_iterations=2000, use_loss=int(use_loss),
                     robust_threshold=3.0, **TOL)
        x = ev.get_params()
    assert np.isclose(s["initial_cost"], s_ref["initial_cost"], rtol=1e-11)
    assert s["num_iterations"] == 1
    m = _free_mask(P)
    assert _close(x[m], x_ref[m], 1e-8), np.abs(x[m] - x_ref[m]).max()
    assert np.array_equal(x[~m], P.params[~m])


@pytest.mark.parametrize("models", [["rpc2", "radtan"], ["rpc3", "fov"], ["rpc4", "radtan"], ["rpc6", "fov"]])
def test_one_exact_step_high_rpc_degree(models):
    """RPC distortion floating, one exact-CG LM step equals the dense step
    (relative 1e-8), focal + distortion floating. Degrees 2 and 3 take pass B's
    register path that folds the distortion columns through the monomials
    (pass_b_rpc_obs: the kNx/kDx/kNy/kDy index mapping of each degree); degrees
    4 and 6 (K = 116 / 220) the wide-row pass B and Gram paths."""
    from oracle import lm_reference

    R = rig.make_rig(num_sensors=len(models), num_ref=10, num_points=250, obs_per_point=5, models=models, seed=97)
    P = rig.build_problem(R, rig.FloatFlags(camera_poses_to_float=(), intrinsics_to_float=("focal_length",
                                                                                           "distortion")))
    x_ref, s_ref = lm_reference.solve(P, max_num_iterations=1, use_loss=True, **TOL)
    with Evaluator(P) as ev:
        assert ev.lin_layout()["supported"]
        ev.set_params()
        s = ev.solve(max_num_iterations=1, eta=1e-14, max_linear_solver_iterations=4000, use_loss=1,
                     robust_threshold=3.0, **TOL)
        x = ev.get_params()
    assert np.isclose(s["initial_cost"], s_ref["initial_cost"], rtol=1e-11)
    m = _free_mask(P)
    assert _close(x[m], x_ref[m], 1e-8), np.abs(x[m] - x_ref[m]).max()


def test_one_exact_step_multiblock_camera_side():
    """Camera side wide enough that the CG vector kernels (k_vec_rep_reduce,
    k_cg_update, 256 entries per block) and the reductions they finalise run on
    many blocks: --no_rig with the non-reference sensors' image poses floating
    (about 2,100 camera-side unknowns = 9 blocks). One exact-CG LM step equals
    the dense step (relative 1e-8), with and without the Cauchy loss."""
    from oracle import lm_reference

    R = rig.make_rig(num_sensors=3, num_ref=150, num_points=1000, obs_per_point=8, models=["radtan", "fov", "none"],
                     seed=91)
    P = rig.build_problem(R, rig.FloatFlags(no_rig=True, camera_poses_to_float=("cam1", "cam2"),
                                            float_timestamp_offsets=False))
    with Evaluator(P) as ev:
        ng = ev.lin_layout()["cam_grad_size"]
    assert ng > 8 * 256, ng
    for use_loss in (False, True):
        x_ref, s_ref = lm_reference.solve(P, max_num_iterations=1, use_loss=use_loss, **TOL)
        with Evaluator(P) as ev:
            ev.set_params()
            s = ev.solve(max_num_iterations=1, eta=1e-14, max_linear_solver_iterations=4000, use_loss=int(use_loss),
                         robust_threshold=3.0, **TOL)
            x = ev.get_params()
        assert np.isclose(s["initial_cost"], s_ref["initial_cost"], rtol=1e-11)
        assert s["num_iterations"] == 1
        m = _free_mask(P)
        assert _close(x[m], x_ref[m], 1e-8), (use_loss, np.abs(x[m] - x_ref[m]).max())


def test_camera_side_past_1024_blocks():
    """More than 1024 blocks' worth of camera-side unknowns (--no_rig, every
    image pose floating: about 283k unknowns): the CG kernels' grid reductions
    run with >1024 partials (their partial buffer is sized from the camera
    side). One LM iteration: no failure, and the step removes most of the
    perturbation's cost (the initial values are the truth perturbed by 1 cm /
    0.1 deg poses and 2 cm points)."""
    R = rig.make_rig(num_sensors=3, num_ref=13500, num_points=120000, obs_per_point=10,
                     models=["radtan"] * 3, seed=93, window=12)
    P = rig.build_problem(R, rig.FloatFlags(no_rig=True, camera_poses_to_float=("ref_cam", "cam1", "cam2"),
                                            float_timestamp_offsets=False))
    with Evaluator(P) as ev:
        ng = ev.lin_layout()["cam_grad_size"]
        assert ng > 1024 * 256, ng
        ev.set_params()
        s = ev.solve(max_num_iterations=2, use_loss=1, robust_threshold=3.0, **TOL)
        x = ev.get_params()
    assert s["termination_type"] != 2, s["message"]
    assert s["num_linear_iterations"] > 0 and s["num_successful_steps"] >= 2
    assert s["final_cost"] < 0.2 * s["initial_cost"], (s["initial_cost"], s["final_cost"])
    assert np.all(np.isfinite(x))


def _poses(P, x):
    """Free 7-parameter blocks as (t, q/|q| with qw >= 0): the cost only sees the
    normalized quaternion (array_to_rigid_transform, dense_map_utils.cc:171-178),
    so |q| is a gauge direction the comparison must ignore."""
    out = []
    for b in np.nonzero((P.block_size == 7) & (P.block_constant == 0))[0]:
        o = int(P.block_offset[b])
        q = x[o + 3:o + 7] / np.linalg.norm(x[o + 3:o + 7])
        out.append(np.r_[x[o:o + 3], q * np.sign(q[3])])
    return np.array(out)


def _others(P, x):
    m = np.zeros(x.size, dtype=bool)
    for b in np.nonzero((P.block_size != 7) & (P.block_constant == 0))[0]:
        o = int(P.block_offset[b])
        m[o:o + int(P.block_size[b])] = True
    return x[m]


INTR_ALL = ("focal_length", "optical_center", "distortion")


@pytest.mark.parametrize("models,use_loss,intr", [
    (["radtan", "fov", "none"], False, INTR_ALL),
    (["radtan", "fov", "none"], True, INTR_ALL),
    (["none", "none", "none"], False, INTR_ALL),
    (["rpc2", "rpc2"], True, ("focal_length", "optical_center")),
])
def test_converged_params_match_cpu_lm(models, use_loss, intr):
    """Poses within 1e-6 (north_star) and every other free parameter within 1e-6
    relative of the CPU LM. (Two CPU runs with different initial radii agree to
    ~5e-10 on poses and ~5e-8 elsewhere on these problems.)"""
    from oracle import lm_reference

    R = rig.make_rig(num_sensors=len(models), num_ref=12, num_points=300, obs_per_point=5, models=models,
                     seed=43 + len(models) + int(use_loss))
    P = rig.build_problem(R, rig.FloatFlags(camera_poses_to_float=(), intrinsics_to_float=intr))
    x_ref, s_ref = lm_reference.solve(P, max_num_iterations=100, use_loss=use_loss, **TOL)
    assert s_ref["message"] in ("parameter tolerance", "function tolerance", "gradient tolerance")
    with Evaluator(P) as ev:
        ev.set_params()
        s = ev.solve(max_num_iterations=200, use_loss=int(use_loss), robust_threshold=3.0, **TOL)
        x = ev.get_params()
    assert s["termination_type"] == 0, s["message"]
    assert s["final_cost"] < s["initial_cost"]
    assert np.isclose(s["final_cost"], s_ref["final_cost"], rtol=1e-9)
    assert np.abs(_poses(P, x) - _poses(P, x_ref)).max() <= 1e-6
    assert _close(_others(P, x), _others(P, x_ref), 1e-6)


def test_c1_converged_params_match_cpu_lm():
    """BASELINE config c1 whole (3 sensors, 1k landmarks / ~5k observations,
    pinhole): converged poses within 1e-6 of the CPU LM (north_star), other
    free parameters within 1e-6 relative, same final cost (the CPU LM takes its
    sparse exact-step path at this size)."""
    from oracle import lm_reference

    R = rig.make_rig(**rig.CONFIGS["c1"])
    P = rig.build_problem(R, rig.FloatFlags(camera_poses_to_float=(), intrinsics_to_float=("focal_length",)))
    x_ref, s_ref = lm_reference.solve(P, max_num_iterations=100, use_loss=True, **TOL)
    assert s_ref["message"] in ("parameter tolerance", "function tolerance", "gradient tolerance")
    with Evaluator(P) as ev:
        ev.set_params()
        s = ev.solve(max_num_iterations=200, use_loss=1, robust_threshold=3.0, **TOL)
        x = ev.get_params()
    assert s["termination_type"] == 0, s["message"]
    assert s["final_cost"] < s["initial_cost"]
    assert np.isclose(s["final_cost"], s_ref["final_cost"], rtol=1e-9)
    assert np.abs(_poses(P, x) - _poses(P, x_ref)).max() <= 1e-6
    assert _close(_others(P, x), _others(P, x_ref), 1e-6)


def test_ill_conditioned_rpc_reaches_same_cost():
    """RPC distortion floated with focal and center is ill-conditioned: the RPC
    terms absorb part of that sensor's rig rotation, so two CPU runs with
    different initial radii end ~1e-3 apart in RPC coefficients at costs equal to
    1e-12, and the GPU run ends 1e-3 apart in that rig quaternion. Parameters are
    not determined there; require the same final cost (rtol 1e-9)."""
    from oracle import lm_reference

    R = rig.make_rig(num_sensors=3, num_ref=12, num_points=300, obs_per_point=5,
                     models=["radtan", "fov", "rpc1"], seed=43)
    P = rig.build_problem(R, FLAGS)
    x_ref, s_ref = lm_reference.solve(P, max_num_iterations=100, **TOL)
    with Evaluator(P) as ev:
        ev.set_params()
        s = ev.solve(max_num_iterations=200, **TOL)
        x = ev.get_params()
    assert s["termination_type"] == 0, s["message"]
    assert np.isclose(s["final_cost"], s_ref["final_cost"], rtol=1e-9)
    assert np.all(np.isfinite(x))


DEPTH_FLAGS = dict(camera_poses_to_float=(), depth_tri_weight=10.0, depth_to_image_transforms_to_float=("cam2",),
                   float_scale=True)


@pytest.mark.parametrize("affine", [False, True])
def test_depth_one_exact_step_matches_dense_lm(affine):
    """BracketedDepthError blocks in the implicit Schur product, right-hand side
    and back-substitution: one exact-CG LM step equals the dense step."""
    from oracle import lm_reference

    R = rig.make_rig(num_sensors=3, num_ref=12, num_points=200, obs_per_point=5, models=["radtan", "fov", "none"],
                     seed=81, depth_sensors=(2,), affine_depth=affine)
    P = rig.build_problem(R, rig.FloatFlags(affine_depth_to_image=affine, **DEPTH_FLAGS))
    assert P.num_depth_residuals > 0
    for use_loss in (False, True):
        x_ref, s_ref = lm_reference.solve(P, max_num_iterations=1, use_loss=use_loss, **TOL)
        with Evaluator(P) as ev:
            ev.set_params()
            s = ev.solve(max_num_iterations=1, eta=1e-14, max_linear_solver_iterations=2000, use_loss=int(use_loss),
                         robust_threshold=3.0, **TOL)
            x = ev.get_params()
        assert np.isclose(s["initial_cost"], s_ref["initial_cost"], rtol=1e-11)
        m = _free_mask(P)
        assert _close(x[m], x_ref[m], 1e-8), (use_loss, np.abs(x[m] - x_ref[m]).max())


def test_depth_converged_params_match_cpu_lm():
    from oracle import lm_reference

    R = rig.make_rig(num_sensors=3, num_ref=12, num_points=200, obs_per_point=5, models=["radtan", "fov", "none"],
                     seed=82, depth_sensors=(2,))
    P = rig.build_problem(R, rig.FloatFlags(**DEPTH_FLAGS))
    x_ref, s_ref = lm_reference.solve(P, max_num_iterations=100, use_loss=True, **TOL)
    with Evaluator(P) as ev:
        ev.set_params()
        s = ev.solve(max_num_iterations=200, use_loss=1, robust_threshold=3.0, **TOL)
        x = ev.get_params()
    assert s["termination_type"] == 0, s["message"]
    assert np.isclose(s["final_cost"], s_ref["final_cost"], rtol=1e-9)
    assert np.abs(_poses(P, x) - _poses(P, x_ref)).max() <= 1e-6
    assert _close(_others(P, x), _others(P, x_ref), 1e-6)


def test_bounded_offsets_and_callback_path():
    """Floated timestamp offsets carry the reference's bracket bounds; a no-op
    allreduce callback (single rank: the sharded code path, exchange, then
    damping and dot as separate kernels) reaches the same solution. The camera
    side adds shared blocks with fp64 atomics, so two solves agree to rounding,
    not bit for bit (bit-identity: the deterministic mode, below)."""
    R, P = _problem(["radtan", "radtan", "fov"], seed=55)
    lo, hi = rig.offset_bounds(R, P, FLAGS)
    assert np.isfinite(lo).sum() == 2
    calls = []
    with Evaluator(P) as ev:
        ev.set_params()
        s0 = ev.solve(max_num_iterations=100, lower_bounds=lo, upper_bounds=hi, **TOL)
        x0 = ev.get_params()
        ev.set_params()
        s1 = ev.solve(max_num_iterations=100, lower_bounds=lo, upper_bounds=hi,
                      allreduce=lambda ptr, n, op: calls.append((n, op)), **TOL)
        x1 = ev.get_params()
    assert calls and all(op in (0, 1) for _, op in calls)
    assert s0["termination_type"] == 0 and s1["termination_type"] == 0
    assert np.isclose(s0["final_cost"], s1["final_cost"], rtol=1e-10)
    # |q| is a gauge direction of the cost (see _poses): compare normalised poses
    assert np.abs(_poses(P, x0) - _poses(P, x1)).max() <= 1e-7
    assert _close(_others(P, x0), _others(P, x1), 1e-7)
    assert np.all(x0 >= lo) and np.all(x0 <= hi)


def test_legacy_three_arg_callback_host_roundtrip():
    """A 3-argument allreduce callback (the pre-stream-ordered contract) reads
    the device buffer to the host and writes it back. The wrapper drains the
    solver's stream before calling it, so the round trip sees finished data and
    the solve reaches the same point as the unsharded one."""
    from multiview_amd.dist import _hip

    R, P = _problem(["radtan", "radtan", "fov"], seed=56)
    hip = _hip()

    def roundtrip(ptr, n, op):
        host = np.empty(n, dtype=np.float64)
        assert hip.hipMemcpy(host.ctypes.data, ptr, 8 * n, 2) == 0
        assert np.all(np.isfinite(host))
        assert hip.hipMemcpy(ptr, host.ctypes.data, 8 * n, 1) == 0

    with Evaluator(P) as ev:
        ev.set_params()
        s0 = ev.solve(max_num_iterations=100, **TOL)
        x0 = ev.get_params()
        ev.set_params()
        s1 = ev.solve(max_num_iterations=100, allreduce=roundtrip, **TOL)
        x1 = ev.get_params()
    assert s0["termination_type"] == 0 and s1["termination_type"] == 0
    assert np.isclose(s0["final_cost"], s1["final_cost"], rtol=1e-10)
    assert np.abs(_poses(P, x0) - _poses(P, x1)).max() <= 1e-7


def test_solver_rejects_bad_options():
    from multiview_amd._lib import MvbaError

    _, P = _problem(["radtan"], seed=60, num_points=50)
    with Evaluator(P) as ev:
        with pytest.raises(MvbaError):
            ev.solve()  # parameters not set
        ev.set_params()
        with pytest.raises(MvbaError):
            ev.solve(use_loss=1, robust_threshold=0.0)
        with pytest.raises(MvbaError):
            ev.solve(max_linear_solver_iterations=0)


# ---------------------------------------------------------------- sharded solve
CFG = dict(num_sensors=3, num_ref=12, num_points=400, obs_per_point=5, models=["radtan", "fov", "none"], seed=77)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cam_values(ev, P):
    """Camera-side blocks in layout order, quaternions normalized (qw >= 0)."""
    L = ev.lin_layout()
    out = []
    for b in L["cam_block_ids"]:
        v = P.block_values(int(b)).copy()
        if v.size == 7:
            v[3:] = v[3:] / np.linalg.norm(v[3:]) * np.sign(v[6])
        out.append(v)
    return np.concatenate(out)


def _points_by_block(ev, P):
    """Point values in parameter-block order (the library numbers points by first
    use in device order; block ids follow the landmark index)."""
    ids = np.sort(ev.lin_layout()["point_block_ids"])
    return np.concatenate([P.block_values(int(b)) for b in ids if b >= 0])


def _shard_worker(rank, world, port, out_dir):
    import sys

    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from multiview_amd.dist import SolverExchange, check_layouts_agree, shard_range

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(CFG["num_points"], world, rank)
    R = rig.make_rig(**dict(CFG, point_range=(lo, hi)))
    P = rig.build_problem(R, FLAGS)
    with Evaluator(P, device=0) as ev:
        check_layouts_agree(ev.lin_layout(), P.block_size)
        ev.set_params()
        ex = SolverExchange()
        s = ev.solve(max_num_iterations=100, allreduce=ex, **TOL)
        P.params = ev.get_params()
        cam = _cam_values(ev, P)
        pts = _points_by_block(ev, P)
    np.save(os.path.join(out_dir, f"cam{rank}.npy"), cam)
    np.save(os.path.join(out_dir, f"pts{rank}.npy"), pts)
    np.save(os.path.join(out_dir, f"cost{rank}.npy"), np.array([s["final_cost"], s["termination_type"]]))
    dist.barrier()
    dist.destroy_process_group()


def _union_problem(world):
    """The unsharded problem = union of the shards' landmarks (point order: first
    use in residual order = shard 0's points, then shard 1's, ...)."""
    from multiview_amd.dist import shard_range

    parts = [rig.make_rig(**dict(CFG, point_range=shard_range(CFG["num_points"], world, r))) for r in range(world)]
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
    return rig.build_problem(R0, FLAGS)


def test_sharded_solve_matches_unsharded(tmp_path):
    import torch.multiprocessing as mp

    from multiview_amd.dist import shard_range

    world = 2
    mp.spawn(_shard_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    cams = [np.load(tmp_path / f"cam{r}.npy") for r in range(world)]
    pts = np.concatenate([np.load(tmp_path / f"pts{r}.npy") for r in range(world)])
    costs = [np.load(tmp_path / f"cost{r}.npy") for r in range(world)]
    assert np.array_equal(cams[0], cams[1])
    assert costs[0][1] == 0 and costs[0][0] == costs[1][0]
    P = _union_problem(world)
    with Evaluator(P) as ev:
        ev.set_params()
        s = ev.solve(max_num_iterations=100, **TOL)
        P.params = ev.get_params()
        cam = _cam_values(ev, P)
        pts_ref = _points_by_block(ev, P)
    assert s["termination_type"] == 0
    assert np.isclose(costs[0][0], s["final_cost"], rtol=1e-9)
    assert _close(cams[0], cam, 1e-6)
    # points by block id = landmark order: shard 0's landmarks, then shard 1's
    assert _close(pts, pts_ref, 1e-6)


def test_local_comm_sharded_solve_device_resident():
    """Two landmark shards in ONE process, one thread and one HIP stream each,
    both on cuda:0, exchanging through the library's local communicator
    (mvba_comm_init_local + mvba_comm_allreduce: stream-ordered device
    all-reduce, no host staging). The device CG runs in sharded mode; both
    shards end with bit-identical camera blocks, and the result equals the
    unsharded solve."""
    import threading

    import torch

    from multiview_amd.dist import Comm, shard_range

    world = 2
    comms = Comm.local([0] * world)
    evs, probs = [], []
    for r in range(world):
        R = rig.make_rig(**dict(CFG, point_range=shard_range(CFG["num_points"], world, r)))
        P = rig.build_problem(R, FLAGS)
        ev = Evaluator(P, device=0)
        ev.set_params()
        evs.append(ev)
        probs.append(P)
    streams = [torch.cuda.Stream() for _ in range(world)]
    out = [None] * world
    errs = []

    def run(r):
        try:
            out[r] = evs[r].solve(max_num_iterations=100, comm=comms[r], stream=streams[r].cuda_stream, **TOL)
        except Exception as e:  # noqa: BLE001
            errs.append(e)
            comms[r].abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    torch.cuda.synchronize()
    cams, pts = [], []
    for r in range(world):
        probs[r].params = evs[r].get_params()
        cams.append(_cam_values(evs[r], probs[r]))
        pts.append(_points_by_block(evs[r], probs[r]))
    assert out[0]["termination_type"] == 0, out[0]["message"]
    assert out[0]["final_cost"] == out[1]["final_cost"]
    assert out[0]["num_linear_iterations"] == out[1]["num_linear_iterations"]
    assert np.array_equal(cams[0], cams[1])
    for ev in evs:
        ev.close()
    for c in comms:
        c.close()
    P = _union_problem(world)
    with Evaluator(P) as ev:
        ev.set_params()
        s = ev.solve(max_num_iterations=100, **TOL)
        P.params = ev.get_params()
        cam = _cam_values(ev, P)
        pts_ref = _points_by_block(ev, P)
    assert np.isclose(out[0]["final_cost"], s["final_cost"], rtol=1e-9)
    assert _close(cams[0], cam, 1e-6)
    assert _close(np.concatenate(pts), pts_ref, 1e-6)


def _rccl_world1_worker(port, out):
    """One rank: torch.distributed over RCCL (world 1), the library's RCCL
    communicator joined from the broadcast unique id (dist.Comm.rccl, the path
    bench.py takes at N > 1), a solve exchanging through it."""
    import os

    import torch
    import torch.distributed as dist

    from multiview_amd.dist import Comm

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    try:
        comm = Comm.rccl(0)
        P = rig.build_problem(rig.make_rig(**CFG), FLAGS)
        with Evaluator(P) as ev:
            ev.set_params()
            s = ev.solve(max_num_iterations=100, comm=comm, **TOL)
            np.save(out, ev.get_params())
            np.save(out + ".cost.npy", np.array([s["final_cost"], s["termination_type"]]))
        comm.close()
    finally:
        dist.destroy_process_group()


def test_rccl_comm_world1_solve(tmp_path):
    """mvba_comm_init_rccl + mvba_comm_allreduce (RCCL) at world size 1 in a
    child process: the communicator bench.py builds for N > 1 initialises from
    the torch.distributed-broadcast unique id, and a solve exchanging through it
    converges to the unsharded solve's point (the exchange is an identity at
    world 1, so only the plumbing is under test). Both solves run to
    convergence, like the sharded tests: the RCCL run takes the sharded
    product form (p.q exchanged with the product) and the single-rank one the
    atomic p.q, so their truncated CG steps differ by rounding, and a
    comparison after 20 LM iterations (not yet converged) compares two points
    of two trajectories (r05t, with a third p.q form: points > 1e-6 apart)."""
    import multiprocessing as mpc
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "rccl_params.npy")
    ctx = mpc.get_context("spawn")
    p = ctx.Process(target=_rccl_world1_worker, args=(port, out))
    p.start()
    p.join(240)
    if p.is_alive():  # never leave a rank holding the GPU behind
        p.kill()
        p.join()
    assert p.exitcode == 0, p.exitcode
    P = rig.build_problem(rig.make_rig(**CFG), FLAGS)
    with Evaluator(P) as ev:
        ev.set_params()
        s_ref = ev.solve(max_num_iterations=100, **TOL)
        P.params = ev.get_params()
        cam, pts = _cam_values(ev, P), _points_by_block(ev, P)
        P.params = np.load(out)
        cam_r, pts_r = _cam_values(ev, P), _points_by_block(ev, P)
    cost, term = np.load(out + ".cost.npy")
    assert int(term) == s_ref["termination_type"] == 0
    assert np.isclose(cost, s_ref["final_cost"], rtol=1e-9)
    # same tolerances as the sharded tests (normalised poses: |q| is a gauge direction)
    assert _close(cam_r, cam, 1e-6)
    assert _close(pts_r, pts, 1e-6)


def test_invalid_step_skips_candidate_range_check(monkeypatch):
    """Ceres rejects an invalid step (non-positive or NaN model change, CG
    failure) without evaluating its candidate, so the reference's
    interpolation check (LOG(FATAL), rig_calibrator.cc:346) never sees that
    candidate. The merged LM step evaluates the candidate speculatively; its
    device error must count only for a valid step, so both read paths
    (MVBA_LM_MERGED=1 / 0) end the same way.

    Rig: sensor 1's images are generated at alpha + 1 (extrapolated past their
    brackets; make_rig alpha_shift), so the offset that explains the data lies
    outside the bracket and the first LM step's candidate leaves [0, 1] (the
    floated offset carries no bounds here). (1) A valid first step raises
    MVBA_E_ALPHA_RANGE in both modes. (2) With the first step declared invalid
    (MVBA_TEST_INVALID_STEPS=1, after its model change is known) and one LM
    iteration, both modes return the same summary: no error, the step counted
    unsuccessful, the parameters unchanged."""
    from multiview_amd import _lib

    R = rig.make_rig(num_sensors=2, num_ref=10, num_points=200, obs_per_point=5, models=["radtan", "fov"], seed=61,
                     alpha_shift=1.0)
    P = rig.build_problem(R, rig.FloatFlags(camera_poses_to_float=()))
    kw = dict(max_num_iterations=1, use_loss=1, robust_threshold=3.0, deterministic=1, **TOL)
    for merged in ("1", "0"):
        monkeypatch.setenv("MVBA_LM_MERGED", merged)
        with Evaluator(P) as ev:
            ev.set_params()
            with pytest.raises(_lib.MvbaError) as e:
                ev.solve(**kw)
            assert e.value.status == _lib.MVBA_E_ALPHA_RANGE, (merged, e.value)
    out = {}
    monkeypatch.setenv("MVBA_TEST_INVALID_STEPS", "1")
    for merged in ("1", "0"):
        monkeypatch.setenv("MVBA_LM_MERGED", merged)
        with Evaluator(P) as ev:
            ev.set_params()
            s = ev.solve(**kw)
            x = ev.get_params()
        assert s["termination_type"] == 1, (merged, s["message"])  # NO_CONVERGENCE: iteration cap
        assert s["num_unsuccessful_steps"] == 1 and s["num_successful_steps"] == 1, (merged, s)
        assert s["final_cost"] == s["initial_cost"]
        assert np.array_equal(x, P.params), merged
        out[merged] = s
    for k in ("termination_type", "num_iterations", "num_successful_steps", "num_unsuccessful_steps",
              "num_linear_iterations", "initial_cost", "final_cost"):
        assert out["1"][k] == out["0"][k], (k, out["1"][k], out["0"][k])
