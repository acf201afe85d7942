"""Deterministic mode (mvba_solver_options.deterministic, MVBA_LIN_DETERMINISTIC).

The default solve adds the camera-side entries shared by many frames (a sensor's
extrinsics and intrinsics) with fp64 atomics into replicas, so rounding depends
on arrival order and the eta = 0.1 truncated CG reacts to it (the reference's
own note, rig_calibrator.cc:1913: "The result is more predictable with one
thread"). Deterministic mode stores every contribution in its producer's slab
row and sums each entry in a fixed order.

Checked here: two deterministic linearizations / solves are bit-identical
(normal equations; CG counts, costs and parameters); the deterministic normal
equations equal the oracle's J^T r / J_b^T J_b (1e-9, as tests/test_linearize_gpu.py)
and agree with the atomic path to rounding; the deterministic and the default (atomic) solves each converge
to the CPU LM's minimum (1e-6, the north_star tolerance); captured CG runs
replay the eager launches bit for bit, single-rank and through a one-rank RCCL
communicator (the sharded path, with the all-reduce inside the graph)."""
import numpy as np
import pytest
import torch

from multiview_amd import rig
from multiview_amd.evaluator import Evaluator
from oracle.normal_equations import normal_equations_reference

pytestmark = pytest.mark.gpu

TOL = dict(function_tolerance=1e-16, gradient_tolerance=1e-16, parameter_tolerance=1e-12)


def _rig_problem(depth=False, num_points=2000, num_ref=40, seed=5, models=("radtan", "rpc2", "fov")):
    kw = dict(depth_sensors=(2,)) if depth else {}
    R = rig.make_rig(num_sensors=3, num_ref=num_ref, num_points=num_points, obs_per_point=6,
                     models=list(models), seed=seed, **kw)
    F = rig.FloatFlags(camera_poses_to_float=(), intrinsics_to_float=("focal_length", "optical_center",
                                                                       "distortion"),
                       **(dict(depth_tri_weight=10.0, depth_to_image_transforms_to_float=("cam2",), float_scale=True)
                          if depth else {}))
    return rig.build_problem(R, F)


def _linearize(ev, det):
    L = ev.lin_layout()
    t = lambda n: torch.zeros(max(n, 1), dtype=torch.float64, device="cuda")  # noqa: E731
    g, h, pg, ph, c = t(L["cam_grad_size"]), t(L["cam_hess_size"]), t(3 * L["num_points"]), \
        t(6 * L["num_points"]), t(1)
    ev.linearize_device(g, h, pg, ph, c, apply_loss=True, robust_threshold=3.0, deterministic=det)
    ev.sync()
    return [x.cpu().numpy() for x in (g, h, pg, ph, c)]


@pytest.mark.parametrize("depth", [False, True])
def test_deterministic_normal_equations(depth, oracle):
    P = _rig_problem(depth)
    with Evaluator(P) as ev:
        ev.set_params()
        a = _linearize(ev, True)
        b = _linearize(ev, True)
        c = _linearize(ev, False)
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
        for x, y in zip(a, c):
            assert np.allclose(x, y, rtol=1e-12, atol=1e-12 * max(1.0, np.abs(y).max()))
        if not depth:
            _, r_o, J_o = oracle.evaluate(P, oracle.ANALYTIC, apply_loss=True, robust_threshold=3.0)
            g_ref, h_ref, _, _ = normal_equations_reference(P, r_o, J_o, ev.lin_layout())
            assert np.abs(a[0][:g_ref.size] - g_ref).max() <= 1e-9 * max(1.0, np.abs(g_ref).max())
            assert np.abs(a[1][:h_ref.size] - h_ref).max() <= 1e-9 * max(1.0, np.abs(h_ref).max())


@pytest.mark.parametrize("depth", [False, True])
def test_deterministic_solve_is_reproducible(depth):
    # RPC coefficients floated with focal and centre are ill-conditioned (DESIGN.md
    # §4c): the parameter comparison uses well-posed models
    P = _rig_problem(depth, models=("radtan", "fov", "radtan"))
    runs = []
    for _ in range(2):
        with Evaluator(P) as ev:
            ev.set_params()
            s = ev.solve(max_num_iterations=6, use_loss=1, robust_threshold=3.0, deterministic=1, **TOL)
            runs.append((s, ev.get_params()))
    (s0, x0), (s1, x1) = runs
    assert s0["num_linear_iterations"] == s1["num_linear_iterations"]
    assert s0["num_iterations"] == s1["num_iterations"]
    assert s0["final_cost"] == s1["final_cost"]
    assert np.array_equal(x0, x1)


@pytest.mark.parametrize("depth", [False, True])
def test_atomic_and_deterministic_solves_reach_the_cpu_minimum(depth):
    """Both summation orders converge (termination CONVERGENCE) to the minimum
    the CPU LM (oracle/lm_reference.py, exact dense steps) reaches on the same
    problem: final cost rtol 1e-9, poses 1e-6, other free parameters 1e-6
    relative (north_star). Without the Cauchy loss the cost has one basin, so
    a different summation order can change the path (the truncated CG's
    stopping points) but not the end point; with the loss two solves may settle
    in different basins (b39ef2c: 6896.5 vs 6893.7 after 50 iterations), which
    says nothing about either order's correctness."""
    from oracle import lm_reference
    from test_solver_gpu import _others, _poses

    P = _rig_problem(depth, num_points=400, num_ref=16, seed=7, models=("radtan", "fov", "radtan"))
    x_ref, s_ref = lm_reference.solve(P, max_num_iterations=100, use_loss=False, **TOL)
    assert s_ref["message"] in ("parameter tolerance", "function tolerance", "gradient tolerance")
    for det in (0, 1):
        with Evaluator(P) as ev:
            ev.set_params()
            s = ev.solve(max_num_iterations=200, use_loss=0, deterministic=det, **TOL)
            x = ev.get_params()
        assert s["termination_type"] == 0, (det, s["message"])
        assert np.isclose(s["final_cost"], s_ref["final_cost"], rtol=1e-9), (det, s["final_cost"], s_ref["final_cost"])
        # |q| of a floated rigid transform (depth_to_image here) is a gauge
        # direction of the cost: compare normalised poses (tests/test_solver_gpu.py)
        assert np.abs(_poses(P, x) - _poses(P, x_ref)).max() <= 1e-6, det
        o, o_ref = _others(P, x), _others(P, x_ref)
        assert np.abs(o - o_ref).max() <= 1e-6 * max(1.0, np.abs(o_ref).max()), (det, np.abs(o - o_ref).max())


@pytest.mark.parametrize("depth", [False, True])
def test_graph_replayed_cg_equals_eager(monkeypatch, depth):
    """Single-rank solves replay captured runs of CG iterations (hipGraph,
    mvba_solve.cpp cg_device; MVBA_CG_GRAPH=0 launches every kernel eagerly).
    The captured launches are the eager ones with the same arguments, so in
    deterministic mode the two give bit-identical solves: CG counts, costs,
    parameters. Long enough for the residual reset (every 10th iteration) and
    both parities of the double-buffered vectors, with the captured runs
    replayed across several linear solves of one handle."""
    P = _rig_problem(depth)
    runs = []
    for g in ("0", "1"):
        monkeypatch.setenv("MVBA_CG_GRAPH", g)
        with Evaluator(P) as ev:
            ev.set_params()
            s = ev.solve(max_num_iterations=6, use_loss=1, robust_threshold=3.0, deterministic=1, **TOL)
            runs.append((s, ev.get_params()))
    (sa, xa), (sb, xb) = runs
    assert sa["num_linear_iterations"] > 20, sa["num_linear_iterations"]
    for k in ("termination_type", "num_iterations", "num_successful_steps", "num_linear_iterations", "final_cost"):
        assert sa[k] == sb[k], (k, sa[k], sb[k])
    assert np.array_equal(xa, xb)


def test_cg_control_mirror_equals_copy(monkeypatch):
    """Where a batch of CG iterations ended reaches the host through the
    CgMirror the batch's last update launch writes into host-coherent memory
    (mvba_solve.cpp cg_device), or, with MVBA_CG_MIRROR=0 / pipelined batches,
    through a device-to-host copy and an event. The host only decides where
    the next batch starts, so every form gives the same deterministic solve,
    bit for bit, eager and captured; solves whose CG stops inside a batch
    mirror from gated launches too (the stop is not the batch's last
    iteration)."""
    P = _rig_problem(False)
    runs = []
    for env in ({"MVBA_CG_MIRROR": "0"}, {"MVBA_CG_MIRROR": "1"}, {"MVBA_CG_MIRROR": "1", "MVBA_CG_GRAPH": "0"},
                {"MVBA_CG_PIPE": "1"}):
        for k in ("MVBA_CG_MIRROR", "MVBA_CG_GRAPH", "MVBA_CG_PIPE"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        with Evaluator(P) as ev:
            ev.set_params()
            s = ev.solve(max_num_iterations=6, use_loss=1, robust_threshold=3.0, deterministic=1, **TOL)
            runs.append((env, s, ev.get_params()))
    _, s0, x0 = runs[0]
    assert s0["num_linear_iterations"] > 20, s0["num_linear_iterations"]
    for env, s, x in runs[1:]:
        for k in ("termination_type", "num_iterations", "num_successful_steps", "num_linear_iterations",
                  "final_cost"):
            assert s[k] == s0[k], (env, k, s[k], s0[k])
        assert np.array_equal(x, x0), env


@pytest.mark.parametrize("null_stream", [False, True])
def test_rccl_captured_cg_equals_eager(monkeypatch, null_stream):
    """The sharded solve's CG runs are captured with the exchange inside
    (mvba_solve.cpp cg_device: an RCCL communicator's ncclAllReduce is a plain
    enqueue on the solver's stream). Through a one-rank RCCL communicator
    (dist.Comm.rccl_world1: the fold-mode CG tail, p.q exchanged with the
    product), deterministic mode, captured == eager bit for bit, and the
    captured solve did replay graphs (cg_graph_launches > 0). null_stream:
    the caller passes the null stream (as bench.py's LM phase does), and the
    library runs the RCCL-sharded solve on its own capturable stream."""
    from multiview_amd.dist import Comm

    P = _rig_problem(False)
    runs = []
    st = torch.cuda.Stream()  # capturable (the null stream is not)
    comm = Comm.rccl_world1(0)
    try:
        for g in ("0", "1"):
            monkeypatch.setenv("MVBA_CG_GRAPH", g)
            with Evaluator(P) as ev:
                ev.set_params()
                s = ev.solve(max_num_iterations=6, use_loss=1, robust_threshold=3.0, deterministic=1, comm=comm,
                             stream=None if null_stream else st.cuda_stream, **TOL)
                runs.append((s, ev.get_params()))
    finally:
        comm.close()
    (sa, xa), (sb, xb) = runs
    assert sa["cg_graph_launches"] == 0
    assert sb["cg_graph_launches"] > 0, sb
    assert sa["num_linear_iterations"] > 20, sa["num_linear_iterations"]
    for k in ("termination_type", "num_iterations", "num_successful_steps", "num_linear_iterations", "final_cost"):
        assert sa[k] == sb[k], (k, sa[k], sb[k])
    assert np.array_equal(xa, xb)


def test_comm_destroy_drops_its_graphs():
    """A captured CG run holds the RCCL communicator's collective (RCCL keeps
    per-graph resources until the graph is destroyed), so mvba_comm_destroy
    first drops every graph recorded with it (mvba_drop_comm_graphs). The
    handle then solves again through a new communicator, capturing afresh, and
    the deterministic solve is the same bit for bit."""
    from multiview_amd.dist import Comm

    P = _rig_problem(False)
    st = torch.cuda.Stream()
    runs = []
    with Evaluator(P) as ev:
        for _ in range(2):
            comm = Comm.rccl_world1(0)
            try:
                ev.set_params()
                s = ev.solve(max_num_iterations=4, use_loss=1, robust_threshold=3.0, deterministic=1, comm=comm,
                             stream=st.cuda_stream, **TOL)
                runs.append((s, ev.get_params()))
            finally:
                comm.close()  # drops the handle's graphs before the communicator
    (sa, xa), (sb, xb) = runs
    assert sa["cg_graph_launches"] > 0 and sb["cg_graph_launches"] > 0, (sa, sb)
    for k in ("termination_type", "num_iterations", "num_linear_iterations", "final_cost"):
        assert sa[k] == sb[k], (k, sa[k], sb[k])
    assert np.array_equal(xa, xb)
