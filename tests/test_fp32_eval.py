"""fp32-output evaluation (config c5: "fp32 eval, fp64 solve"): the same fp64
arithmetic as the fp64 path with each value rounded once at the store, so the
fp32 planes equal the fp64 planes rounded to float (tolerance: one float ulp,
allowing a different fused-multiply-add contraction between the two template
instantiations). The fp64 planes themselves are pinned against the oracle by
tests/test_parity_gpu.py and tests/test_depth.py. Only slots holding a residual
block are compared: padding slots that share a 128-B line with a frame's last
block hold a copy of it, over 16 slots for fp64 outputs and 32 for fp32."""
import ctypes as C

import numpy as np
import pytest

from multiview_amd import _lib, rig
from multiview_amd.evaluator import Evaluator

pytestmark = pytest.mark.gpu


def _close_to_rounded(f32, f64):
    ref = f64.astype(np.float32)
    ulp = np.spacing(np.abs(ref)).astype(np.float64)
    return np.all(np.abs(f32.astype(np.float64) - ref.astype(np.float64)) <= ulp)


@pytest.mark.parametrize("apply_loss", [False, True])
def test_reprojection_f32_equals_rounded_f64(apply_loss):
    import torch

    R = rig.make_rig(num_sensors=4, num_ref=10, num_points=300, obs_per_point=5,
                     models=["radtan", "rpc2", "fov", "none"], seed=61)
    P = rig.build_problem(R)
    with Evaluator(P) as ev:
        ev.set_params()
        ld = ev.ld
        r64 = torch.zeros((2, ld), dtype=torch.float64, device="cuda")
        j64 = torch.zeros((ev.stride, ld), dtype=torch.float64, device="cuda")
        r32 = torch.zeros((2, ld), dtype=torch.float32, device="cuda")
        j32 = torch.zeros((ev.stride, ld), dtype=torch.float32, device="cuda")
        ev.evaluate_device(True, apply_loss=apply_loss, residuals=r64, jac=j64, ld=ld)
        ev.evaluate_device(True, apply_loss=apply_loss, residuals=r32, jac=j32, ld=ld)
        ev.sync()
        live = np.zeros(ld, dtype=bool)
        live[:ev.num_slots] = ev.order() >= 0
    r32, r64 = r32.cpu().numpy()[:, live], r64.cpu().numpy()[:, live]
    j32, j64 = j32.cpu().numpy()[:, live], j64.cpu().numpy()[:, live]
    assert _close_to_rounded(r32, r64)
    assert _close_to_rounded(j32, j64)
    assert np.count_nonzero(j32) > 0.5 * np.count_nonzero(j64)


def test_depth_f32_equals_rounded_f64():
    import torch

    R = rig.make_rig(num_sensors=3, num_ref=10, num_points=120, obs_per_point=4, seed=62, depth_sensors=(2,))
    P = rig.build_problem(R, rig.FloatFlags(depth_tri_weight=10.0, depth_to_image_transforms_to_float=("cam2",),
                                            float_scale=True))
    with Evaluator(P) as ev:
        ev.set_params()
        ev.evaluate_device(False)  # prep (frame records) for the depth kernels
        dld = (ev.num_depth_slots + 63) // 64 * 64
        out = {}
        for dt in (torch.float64, torch.float32):
            r = torch.zeros((3, dld), dtype=dt, device="cuda")
            J = torch.zeros((_lib.DJAC_ROWS, dld), dtype=dt, device="cuda")
            fn = ev.lib.mvba_evaluate_depth_device_f32 if dt == torch.float32 else ev.lib.mvba_evaluate_depth_device
            _lib.check(fn(ev.h, _lib.EVAL_RESIDUALS | _lib.EVAL_JACOBIAN, 0.0, C.c_void_p(r.data_ptr()),
                          C.c_void_p(J.data_ptr()), dld, None), ev.h)
            ev.sync()
            out[dt] = (r.cpu().numpy(), J.cpu().numpy())
        dorder = np.empty(ev.num_depth_slots, dtype=np.int64)
        _lib.check(ev.lib.mvba_depth_order(ev.h, dorder.ctypes.data), ev.h)
    live = np.zeros(dld, dtype=bool)
    live[:len(dorder)] = dorder >= 0
    out = {dt: (r[:, live], J[:, live]) for dt, (r, J) in out.items()}
    assert _close_to_rounded(out[torch.float32][0], out[torch.float64][0])
    assert _close_to_rounded(out[torch.float32][1], out[torch.float64][1])
