"""The rig_calibrator CLI (multiview_amd/cli).

CPU: gflags-style parsing, parameterValidation's messages
(rig_calibrator.cc:893-955), this build's scope refusals, readRigConfig's
checks (dense_map_utils.cc:940-1057), and image lookup / bracketing
(dense_map_utils.cc:1441-1805) up to the first GPU call.
GPU: end-to-end runs against the oracle's restatement of main()
(oracle/rig_calibrator_ref.py, CPU triangulation + dense LM + flagging on the
same files): the printed residual statistics before the first solve (same
inputs, so equal to the printed 5 digits), and the written outputs
(cameras.txt, rig_config.txt) after converged passes within 1e-6 relative
(north_star: converged poses within 1e-6 of the CPU result).
"""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from multiview_amd import rig, rig_files

CLI = os.path.join(ROOT, "multiview_amd", "cli", "rig_calibrator")


@pytest.fixture(scope="module")
def cli():
    subprocess.run(["make", "-s", "-C", os.path.dirname(CLI)], check=True)
    return CLI


def _run(cli, *args, cwd=None, timeout=600):
    p = subprocess.run([cli, *args], capture_output=True, text=True, cwd=cwd, timeout=timeout)
    return p.returncode, p.stdout, p.stderr


def _dataset(tmp_path, models=("radtan", "fov", "none"), num_ref=8, num_points=150, seed=3, **kw):
    R = rig.make_rig(num_sensors=len(models), num_ref=num_ref, num_points=num_points, obs_per_point=4,
                     models=list(models), seed=seed, **kw)
    dti = None
    if kw.get("depth_sensors"):
        dti = np.tile(np.eye(4), (len(models), 1, 1))
        for s in range(len(models)):  # init depth_to_image (rigid 7-array) as 4x4
            a = R.init["depth_to_image"][s]
            dti[s, :3, :3] = rig.quat_to_mat(a[3:][None])[0]
            dti[s, :3, 3] = a[:3]
    return R, rig_files.write_dataset(R, str(tmp_path / "data"), depth_to_image=dti)


# ---------------------------------------------------------------- CPU
VALIDATION = [
    (["--robust_threshold=0"], "The robust threshold must be positive."),
    (["--bracket_len", "-1"], "Bracket length must be positive."),
    (["--no_nvm_matches"], "Then must set a positive --num_overlaps"),
    (["--timestamp_offsets_max_change=-1"], "The timestamp offsets must be non-negative."),
    (["--min_triangulation_angle=0"], "The min triangulation angle must be positive."),
    (["--depth_tri_weight=-1"], "The depth weight must non-negative."),
    (["--tri_weight=1"], "The triangulation robust threshold must be positive."),
    (["--float_scale", "--affine_depth_to_image"], "should not be used together"),
    (["--no_rig", "--float_timestamp_offsets"], "Cannot float timestamps with option --no_rig."),
    (["--out_dir="], "The output directory was not specified."),
    (["--no_rig", "--use_initial_rig_transforms"], "Cannot use initial rig transforms if not modeling the rig."),
    (["--rig_config="], "Must specify the initial rig configuration via --rig_config."),
    (["--camera_poses=x.txt"], "Cannot specify both --nvm and --camera_poses."),
    (["--mesh_tri_weight=-1"], "The mesh weight must non-negative."),
    (["--depth_mesh_weight=-1"], "The depth mesh weight must non-negative."),
    (["--out_texture_dir=t"], "Cannot project camera images onto a mesh if a mesh was not provided."),
    (["--out_texture_dir=t", "--mesh=m.ply"], "--out_texture_dir (texturing) is outside this build's scope"),
    (["--num_overlaps=3"], "feature detection and matching"),
    (["--device=cpu"], "no CPU compute path"),
]


@pytest.mark.parametrize("extra,msg", VALIDATION)
def test_parameter_validation(cli, tmp_path, extra, msg):
    base = ["--rig_config", "r.txt", "--nvm", "c.nvm", "--out_dir", str(tmp_path)]
    code, out, err = _run(cli, *base, *extra)
    assert code == 1
    assert msg in err, err


def test_flag_syntax(cli):
    code, _, err = _run(cli, "--not_a_flag=1")
    assert code == 1 and "unknown command line flag 'not_a_flag'" in err
    code, _, err = _run(cli, "--num_iterations=abc")
    assert code == 1 and "illegal value 'abc'" in err
    # --noflag form for booleans, then validation order as the reference (out_dir first missing)
    code, _, err = _run(cli, "--nofloat_scale", "--nvm", "x.nvm", "--rig_config", "r.txt")
    assert code == 1 and "The output directory was not specified." in err


def test_rig_config_checks(cli, tmp_path):
    R, info = _dataset(tmp_path)
    txt = open(info["rig_config"]).read()
    bad = tmp_path / "bad.txt"
    bad.write_text(txt.replace("distortion_type: fisheye", "distortion_type: radtan", 1))
    code, _, err = _run(cli, "--rig_config", str(bad), "--nvm", info["nvm"], "--out_dir", str(tmp_path / "o"))
    assert code == 1 and "When there is 1 distortion coefficient, distortion type must be: fisheye" in err
    bad.write_text(txt.replace("sensor_name: ref_cam", "sensor_name: other", 1))
    code, _, err = _run(cli, "--rig_config", str(bad), "--nvm", info["nvm"], "--out_dir", str(tmp_path / "o"))
    assert code == 1 and "The reference sensor must be the first sensor" in err
    bad.write_text(txt.replace("focal_length:", "focal:", 1))
    code, _, err = _run(cli, "--rig_config", str(bad), "--nvm", info["nvm"], "--out_dir", str(tmp_path / "o"))
    assert code == 1 and "Could not read value for: focal_length:" in err
    code, _, err = _run(cli, "--rig_config", info["rig_config"], "--nvm", info["nvm"], "--out_dir",
                        str(tmp_path / "o"), "--intrinsics_to_float", "cam1:zoom")
    assert code == 1 and "Unexpected value when parsing intrinsics to float: zoom" in err


def test_image_lookup_and_bracketing(cli, tmp_path):
    """The bracketing picks, per reference interval and sensor, the image closest
    to the middle; the synthetic rig has exactly one such image per interval
    (none after the last reference image), so the counts are known."""
    R, info = _dataset(tmp_path)
    code, out, err = _run(cli, "--rig_config", info["rig_config"], "--nvm", info["nvm"], "--out_dir",
                          str(tmp_path / "o"), "--calibrator_num_passes", "0")
    for s, name in enumerate(R.sensor_names):
        n = int((R.cam_type == s).sum())
        assert f"Number of images for sensor: {name}: {n}" in out, out
    assert "cam1: [" in out  # allowed offset ranges are printed
    # with no passes nothing reaches the GPU: the outputs are written on the CPU
    assert code == 0, err
    lines = open(tmp_path / "o" / "cameras.txt").read().splitlines()
    assert lines[0] == "# image_file world_to_image_transform" and len(lines) == 1 + len(R.cam_type)
    # a bracket longer than --bracket_len drops every non-reference image
    code, out, err = _run(cli, "--rig_config", info["rig_config"], "--nvm", info["nvm"], "--out_dir",
                          str(tmp_path / "o2"), "--bracket_len", "0.4", "--calibrator_num_passes", "0")
    assert code == 1 and "Could not find images for all sensors" in err


@pytest.mark.parametrize("body,msg", [
    ("element vertex -1\nproperty float x\nproperty float y\nproperty float z\nend_header\n",
     "Bad PLY element count"),
    ("element vertex 3\nproperty float x\nproperty float y\nproperty float z\n"
     "element face 1\nproperty list uchar int vertex_indices\nend_header\n"
     "0 0 0\n1 0 0\n0 1 0\n-1 0 1 2\n", "Bad PLY list count"),
    ("element vertex 3\nproperty float x\nproperty float y\nproperty float z\n"
     "element face 1\nproperty list int int vertex_indices\nend_header\n"
     "0 0 0\n1 0 0\n0 1 0\n2000000000 0 1 2\n", "Bad PLY list count"),
    ("element vertex 3\nproperty float x\nproperty float y\nproperty float z\n"
     "element face 1\nproperty list uchar int vertex_indices\nend_header\n"
     "0 0 0\n1 0 0\n0 1 0\n4 0 1 2 0\n", "Only triangle faces are supported"),
    ("element vertex 3\nproperty float x\nproperty float y\nproperty float z\n"
     "element face 1\nproperty list uchar int vertex_indices\nend_header\n"
     "0 0 0\n1 0 0\n0 1 0\n3 0 1 7\n", "PLY face index out of range"),
])
def test_corrupt_ply_is_a_clean_error(cli, tmp_path, body, msg):
    """--mesh files are read on the host before the first GPU call: a corrupt
    count is reported through the CLI's error path, not a bad_alloc abort."""
    R, info = _dataset(tmp_path)
    ply = tmp_path / "bad.ply"
    ply.write_text("ply\nformat ascii 1.0\n" + body)
    code, out, err = _run(cli, "--rig_config", info["rig_config"], "--nvm", info["nvm"], "--out_dir",
                          str(tmp_path / "o"), "--mesh", str(ply), "--mesh_tri_weight", "1")
    assert code == 1 and msg in err, (code, out, err)


def test_rig_config_round_trip(cli, tmp_path):
    """With no passes and --use_initial_rig_transforms the written rig_config.txt
    holds the configuration read in."""
    R, info = _dataset(tmp_path)
    code, out, err = _run(cli, "--rig_config", info["rig_config"], "--nvm", info["nvm"], "--out_dir",
                          str(tmp_path / "o"), "--calibrator_num_passes", "0", "--use_initial_rig_transforms")
    assert code == 0, err
    a = open(info["rig_config"]).read().split("\n")
    b = open(tmp_path / "o" / "rig_config.txt").read().split("\n")
    assert len(a) == len(b)
    for x, y in zip(a, b):
        tx, ty = x.split(), y.split()
        assert tx[:1] == ty[:1]
        if tx and tx[0] in ("sensor_name:", "distortion_type:", "ref_sensor_name:"):
            assert tx == ty
        elif tx:
            assert np.allclose([float(v) for v in tx[1:]], [float(v) for v in ty[1:]], rtol=1e-12, atol=1e-15), (x, y)


def test_rig_from_camera_poses(cli, tmp_path):
    """calc_rig_using_word_to_cam (rig_calibrator.cc:1186-1266): the rig
    transforms written after zero passes equal the oracle restatement's, and the
    camera poses are the rig-derived ones (calc_world_to_cam_using_rig)."""
    from oracle import rig_calibrator_ref
    from oracle.rig_calibrator_ref import _array_to_rigid

    R, info = _dataset(tmp_path)
    code, out, err = _run(cli, "--rig_config", info["rig_config"], "--nvm", info["nvm"], "--out_dir",
                          str(tmp_path / "o"), "--calibrator_num_passes", "0")
    assert code == 0, err
    ref = rig_calibrator_ref.run(info["rig_config"], info["nvm"], calibrator_num_passes=0)
    rows = _read_rig(tmp_path / "o" / "rig_config.txt")
    for t, r in enumerate(rows):
        Rr, tr = _array_to_rigid(ref["ref_to_cam"][t])
        T = np.array(r["ref_to_sensor_transform"])
        assert np.allclose(T[:9], Rr.reshape(-1), rtol=0, atol=1e-13) and np.allclose(T[9:], tr, atol=1e-13)
    cams = _read_cameras(tmp_path / "o" / "cameras.txt")
    for k, nm in enumerate(ref["image_names"]):
        assert np.allclose(cams[nm], ref["world_to_cam"][k], rtol=0, atol=1e-12)


# ---------------------------------------------------------------- GPU
def _parse_stats(out):
    """Blocks of 'The 25, 50, 75, and 100th percentile residual stats <tag>'."""
    blocks, cur = [], None
    for ln in out.splitlines():
        if ln.startswith("The 25, 50, 75, and 100th percentile residual stats"):
            cur = {}
            blocks.append((ln.rsplit(" ", 2)[-2] + " " + ln.rsplit(" ", 2)[-1], cur))
            continue
        m = re.match(r"^(\S+): ([-0-9.e+]+) ([-0-9.e+]+) ([-0-9.e+]+) ([-0-9.e+]+) \((\d+) residuals\)$", ln)
        if cur is not None and m:
            cur[m.group(1)] = ([float(m.group(k)) for k in range(2, 6)], int(m.group(6)))
        elif cur is not None and ln and not m:
            cur = None
    return blocks


def _read_cameras(path):
    out = {}
    for ln in open(path):
        if ln.startswith("#"):
            continue
        t = ln.split()
        out[t[0]] = np.array([float(v) for v in t[1:]])
    return out


def _read_rig(path):
    rows, cur = [], None
    for ln in open(path):
        t = ln.split()
        if not t:
            continue
        if t[0] == "sensor_name:":
            cur = {"name": t[1]}
            rows.append(cur)
        elif cur is not None:
            cur[t[0].rstrip(":")] = [float(v) for v in t[1:]] if t[0] != "distortion_type:" else t[1]
    return rows


CASES = {
    "rig": dict(flags=dict(rig_transforms_to_float="cam1 cam2",
                           intrinsics_to_float="ref_cam:focal_length cam1:focal_length,distortion cam2:focal_length")),
    "no_rig": dict(flags=dict(no_rig=True, camera_poses_to_float="cam1",
                              intrinsics_to_float="cam1:focal_length,optical_center")),
    "tri_weight": dict(flags=dict(rig_transforms_to_float="cam2", tri_weight=0.5, tri_robust_threshold=0.1,
                                  intrinsics_to_float="cam2:distortion")),
    # floating RPC distortion (undistortion refit after each pass); the RPC's
    # linear terms trade off with focal length and rig rotation, so only the
    # distortion of cam1 floats (a unique minimum to compare)
    "rpc": dict(rig=dict(models=("radtan", "rpc1", "fov"), num_points=400),
                flags=dict(rig_transforms_to_float="cam2", intrinsics_to_float="cam1:distortion")),
    "depth": dict(rig=dict(depth_sensors=(2,)),
                  flags=dict(rig_transforms_to_float="cam1 cam2", depth_tri_weight=10.0,
                             depth_to_image_transforms_to_float="cam2", float_scale=True)),
    # --mesh (PLY icosphere of the sphere-surface scene): meshTriangulations each
    # pass, BracketedDepthMeshError + mesh_tri priors beside the depth blocks
    "mesh": dict(rig=dict(depth_sensors=(2,), surface="sphere", num_ref=30, num_points=300),
                 flags=dict(rig_transforms_to_float="cam1 cam2", depth_tri_weight=10.0, depth_mesh_weight=5.0,
                            mesh_tri_weight=2.0, depth_to_image_transforms_to_float="cam2", float_scale=True)),
    # BASELINE config c1 (configs[0]): 3-sensor rig, 1k landmarks / ~5k
    # observations, pinhole without distortion, the whole rig generator config
    "c1": dict(config="c1",
               flags=dict(rig_transforms_to_float="cam1 cam2",
                          intrinsics_to_float="ref_cam:focal_length cam1:focal_length cam2:focal_length")),
}


def _cli_args(flags):
    args = []
    for k, v in flags.items():
        if isinstance(v, bool):
            args.append(f"--{k}" if v else f"--no{k}")
        else:
            args += [f"--{k}", str(v)]
    return args


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES) + ["rig_2shards"])
def test_cli_matches_oracle_pipeline(cli, tmp_path, name):
    """rig_2shards: the "rig" case with --num_gpus 2 (landmark shards, host
    all-reduce between the solver threads; on a one-GPU box both shards share it)."""
    from oracle import rig_calibrator_ref

    shards = 2 if name.endswith("_2shards") else 1
    name = name.replace("_2shards", "")
    flags = dict(CASES[name]["flags"])
    if "config" in CASES[name]:
        R = rig.make_rig(**rig.CONFIGS[CASES[name]["config"]])
        info = rig_files.write_dataset(R, str(tmp_path / "data"))
    else:
        R, info = _dataset(tmp_path, seed=11 + len(name), **CASES[name].get("rig", {}))
    if "mesh_tri_weight" in flags:
        flags["mesh"] = str(tmp_path / "data" / "mesh.ply")
        rig_files.write_ply(flags["mesh"], *rig.sphere_mesh(5))
    out_dir = tmp_path / "out"
    common = dict(num_iterations=100, parameter_tolerance=1e-12)
    code, out, err = _run(cli, "--rig_config", info["rig_config"], "--nvm", info["nvm"], "--out_dir", str(out_dir),
                          *_cli_args({**flags, **common}), "--save_nvm", "--num_gpus", str(shards))
    assert code == 0, err + out[-3000:]
    ref = rig_calibrator_ref.run(info["rig_config"], info["nvm"], **flags, **common)

    # residual statistics before the first solve: identical inputs
    blocks = _parse_stats(out)
    assert [b[0] for b in blocks] == ["before opt", "after opt"] * 2
    before0 = blocks[0][1]
    exp = {r[0]: (list(r[1:5]), r[5]) for r in ref["stats"][0][0]}
    assert set(before0) == set(exp)
    for k, (v, n) in before0.items():
        assert n == exp[k][1]
        assert np.allclose(v, exp[k][0], rtol=1e-4, atol=1e-9), (k, v, exp[k])

    # outputs after two converged passes
    cams = _read_cameras(out_dir / "cameras.txt")
    assert len(cams) == len(ref["image_names"])
    for k, nm in enumerate(ref["image_names"]):
        got = cams[nm]
        want = ref["world_to_cam"][k]
        assert np.abs(got - want).max() <= 1e-6 * max(1.0, np.abs(want).max()), (nm, got, want)
    rows = _read_rig(out_dir / "rig_config.txt")
    for t, r in enumerate(rows):
        assert abs(r["focal_length"][0] - ref["focal"][t]) <= 1e-6 * ref["focal"][t]
        assert np.allclose(r["optical_center"], ref["center"][t], rtol=1e-6)
        got_d, want_d = np.array(r["distortion_coeffs"]), np.asarray(ref["dist"][t])
        if got_d.size > 5:
            # RPC: compare both halves as models on the image (coefficients of
            # high-degree terms are poorly determined individually; the image
            # corners are barely observed in this small rig): 1e-5 of the half size
            from oracle.rpc_fit_reference import compute_rpc

            g = np.stack(np.meshgrid(np.linspace(-500, 500, 21), np.linspace(-380, 380, 17)), -1).reshape(-1, 2)
            h = got_d.size // 2
            for a, b in ((got_d[:h], want_d[:h]), (got_d[h:], want_d[h:])):
                assert np.abs(compute_rpc(g, a) - compute_rpc(g, b)).max() < 1e-5 * 512
        else:
            assert np.allclose(got_d, want_d, rtol=1e-6, atol=1e-8)
        if not flags.get("no_rig"):
            from oracle.rig_calibrator_ref import _array_to_rigid

            Rr, tr = _array_to_rigid(ref["ref_to_cam"][t])
            T = np.array(r["ref_to_sensor_transform"])
            assert np.allclose(T[:9], Rr.reshape(-1), atol=1e-6) and np.allclose(T[9:], tr, atol=1e-6)
    if flags.get("mesh"):
        assert "depth_mesh_x_m" in before0 and "mesh_tri_x_m" in before0
    if flags.get("depth_tri_weight"):
        assert info["num_clouds"] > 0 and "depth_tri_x_m" in before0
        for t, r in enumerate(rows):
            Rd, td = ref["depth_to_image"][t]
            T = np.array(r["depth_to_image_transform"])
            assert np.allclose(T[:9], Rd.reshape(-1), atol=1e-6) and np.allclose(T[9:], td, atol=1e-6)
    # NVM output: inlier tracks with more than two features
    nvm = open(out_dir / "cameras.nvm").read().split()
    assert nvm[0] == "NVM_V3" and int(nvm[1]) == len(ref["image_names"])
