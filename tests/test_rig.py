"""CPU tests of the synthetic rig and of the problem assembly semantics of
rig_calibrator.cc:1614-1752."""
import numpy as np

from multiview_amd import rig
from multiview_amd.problem import distortion_size_valid


def test_rig_is_deterministic():
    a = rig.make_rig(**rig.CONFIGS["c1"])
    b = rig.make_rig(**rig.CONFIGS["c1"])
    assert np.array_equal(a.obs_pix, b.obs_pix)
    assert np.array_equal(a.init["xyz"], b.init["xyz"])


def test_alpha_in_range_and_measurements_float32():
    R = rig.make_rig(**rig.CONFIGS["c1"])
    P = rig.build_problem(R)
    sb, se, sc = P.residual_stamps.T
    off = P.params[P.block_offset[P.residual_blocks[:, 4]]]
    interp = sb != se
    alpha = ((sc[interp] - sb[interp]) - off[interp]) / (se[interp] - sb[interp])
    assert np.all((alpha >= 0) & (alpha <= 1))
    assert np.array_equal(P.residual_meas, P.residual_meas.astype(np.float32).astype(np.float64))


def test_problem_assembly_rules():
    R = rig.make_rig(num_sensors=3, num_ref=20, num_points=200, obs_per_point=4, seed=3)
    flags = rig.FloatFlags(camera_poses_to_float=("ref_cam",), rig_transforms_to_float=("cam1",),
                           intrinsics_to_float=("focal_length",), float_timestamp_offsets=True)
    P = rig.build_problem(R, flags)
    blk, const = P.residual_blocks, P.block_constant
    ref = P.residual_camera == 0
    # end block is the identity placeholder for ref-type observations (:1642-1643)
    assert len(set(blk[ref, 1])) == 1 and const[blk[ref, 1][0]] == 1
    # ref_to_cam is constant for the ref sensor and for sensors not listed (:1749-1752)
    assert np.all(const[blk[P.residual_camera == 0, 2]] == 1)
    assert np.all(const[blk[P.residual_camera == 1, 2]] == 0)
    assert np.all(const[blk[P.residual_camera == 2, 2]] == 1)
    # offsets float only for non-ref sensors (:1737-1746)
    assert np.all(const[blk[ref, 4]] == 1) and np.all(const[blk[~ref, 4]] == 0)
    # intrinsics per --intrinsics_to_float (:1702-1710)
    assert np.all(const[blk[:, 5]] == 0) and np.all(const[blk[:, 6]] == 1) and np.all(const[blk[:, 7]] == 1)
    # residual order: pid-major, then cid (std::map iteration)
    key = R.obs_pid * 10 ** 7 + R.obs_cid
    assert np.all(np.diff(key) > 0)


def test_no_rig_assembly():
    R = rig.make_rig(num_sensors=2, num_ref=10, num_points=100, obs_per_point=4, seed=4)
    P = rig.build_problem(R, rig.FloatFlags(no_rig=True, camera_poses_to_float=("ref_cam", "cam1"),
                                            float_timestamp_offsets=False))
    sb, se, sc = P.residual_stamps.T
    assert np.all(sb == se) and np.all(se == sc)
    assert np.all(P.block_constant[P.residual_blocks[:, 4]] == 1)


def test_distortion_sizes():
    assert [k for k in range(0, 80) if distortion_size_valid(k)] == [0, 1, 4, 5, 20, 44, 76]


def test_shards_partition_points():
    full = rig.make_rig(num_sensors=2, num_ref=10, num_points=100, obs_per_point=4, seed=9,
                        point_range=(0, 100))
    a = rig.make_rig(num_sensors=2, num_ref=10, num_points=100, obs_per_point=4, seed=9,
                     point_range=(0, 50))
    b = rig.make_rig(num_sensors=2, num_ref=10, num_points=100, obs_per_point=4, seed=9,
                     point_range=(50, 100))
    # cameras identical on every shard
    assert np.array_equal(a.init["world_to_ref"], b.init["world_to_ref"])
    assert np.array_equal(full.init["world_to_ref"], a.init["world_to_ref"])
    assert a.xyz.shape[0] == 50 and b.xyz.shape[0] == 50


def test_capture_order_shards_partition_the_problem():
    """rig.shard_points (bench.py's strong split): the shards partition the
    landmarks and observations of the whole problem exactly (same pixels, same
    images, pid-major order), balance the observation count, keep depth
    observations attached to theirs, and each shard sees a stretch of the
    trajectory: far fewer images than the whole problem."""
    R = rig.make_rig(num_sensors=4, num_ref=200, num_points=4000, obs_per_point=6.0, seed=5,
                     models=["radtan"] * 4, depth_sensors=(3,))
    world = 4
    shards = [rig.shard_points(R, r, world) for r in range(world)]
    assert sum(len(S.xyz) for S in shards) == len(R.xyz)
    assert sum(len(S.obs_pid) for S in shards) == len(R.obs_pid)
    assert sum(len(S.depth_obs) for S in shards) == len(R.depth_obs)
    whole = {(tuple(R.xyz[p]), c, tuple(x)) for p, c, x in zip(R.obs_pid, R.obs_cid, R.obs_pix)}
    got = set()
    for S in shards:
        assert np.all(np.diff(S.obs_pid) >= 0)
        assert np.array_equal(S.init["world_to_ref"], R.init["world_to_ref"])
        assert abs(len(S.obs_pid) - len(R.obs_pid) / world) < 0.02 * len(R.obs_pid)
        assert len(np.unique(S.obs_cid)) < 0.5 * len(R.cam_type)
        got |= {(tuple(S.xyz[p]), c, tuple(x)) for p, c, x in zip(S.obs_pid, S.obs_cid, S.obs_pix)}
        # the depth point travels with its observation
        src = {(tuple(R.xyz[R.obs_pid[o]]), R.obs_cid[o]): tuple(m) for o, m in zip(R.depth_obs, R.depth_meas)}
        for o, m in zip(S.depth_obs, S.depth_meas):
            assert src[(tuple(S.xyz[S.obs_pid[o]]), S.obs_cid[o])] == tuple(m)
        rig.build_problem(S)
    assert got == whole
