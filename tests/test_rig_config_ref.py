"""The CLI's rig_config.txt writer pinned by the reference's own parser.

tests/golden/rig_config_ref_parse.json holds, per case, the rig_config.txt the
rig_calibrator CLI wrote (zero passes: read, bracket, write) and what the
reference's ``parseRigConfig`` (rig_calibrator/bin/rig_utils.py:84-185) reads
from it and from the input configuration; tests/golden/make_rig_config_golden.py
made them in the build container. Here (CPU, no reference needed):
  * the CLI, run again on the regenerated dataset, writes the same bytes the
    reference parser was run on;
  * the reference parser read every field of the CLI's output in its order and
    count, and the values equal the input configuration's: names, types and
    sizes as strings, intrinsics / distortion / offsets as the same doubles
    (precision 17 round trip), depth_to_image_transform and (where the rig is
    kept, --use_initial_rig_transforms) ref_to_sensor_transform to 1e-15
    (rotation matrix -> quaternion -> rotation matrix inside the CLI).
"""
import json
import os
import sys

import numpy as np
import pytest

from conftest import ROOT

GOLD = os.path.join(ROOT, "tests", "golden", "rig_config_ref_parse.json")
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

EXACT_STR = ("sensor_name", "distortion_type", "image_size", "distorted_crop_size", "undistorted_image_size")
EXACT_NUM = ("focal_length", "optical_center", "distortion_coeffs", "ref_to_sensor_timestamp_offset")


def _cases():
    with open(GOLD) as f:
        return json.load(f)["cases"]


@pytest.fixture(scope="module")
def cli():
    import subprocess

    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "multiview_amd", "cli")], check=True)


@pytest.mark.parametrize("name", list(_cases()))
def test_cli_rig_config_matches_reference_parse(cli, tmp_path, name):
    from make_rig_config_golden import make_case

    g = _cases()[name]
    _, written = make_case(g["case"], str(tmp_path))
    assert open(written).read() == g["written_text"]
    pw, pi = g["parsed_written"], g["parsed_input"]
    assert len(pw) == len(pi) == len(g["case"]["rig"]["models"])
    for a, b in zip(pw, pi):
        for k in EXACT_STR:
            assert a[k] == b[k], k
        for k in EXACT_NUM:
            va = np.atleast_1d(np.array(a[k], dtype=float))
            vb = np.atleast_1d(np.array(b[k], dtype=float))
            assert va.shape == vb.shape and np.array_equal(va, vb), (k, a[k], b[k])
        D = np.array(a["depth_to_image_transform"], dtype=float)
        assert D.shape == (12,)
        assert np.allclose(D, np.array(b["depth_to_image_transform"], dtype=float), rtol=0, atol=1e-15)
        T = np.array(a["ref_to_sensor_transform"], dtype=float)
        assert T.shape == (12,)
        R = T[:9].reshape(3, 3)
        assert np.abs(R @ R.T - np.eye(3)).max() < 1e-14
        if "--use_initial_rig_transforms" in g["case"]["args"]:
            assert np.allclose(T, np.array(b["ref_to_sensor_transform"], dtype=float), rtol=0, atol=1e-15)
