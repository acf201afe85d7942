#!/usr/bin/env python3
"""Fixtures that pin the CLI's cameras.txt writer (saveCameraPoses,
dense_map_utils.cc:753-776) against the reference's own Python reader,
``parse_images_and_camera_poses`` in
/root/reference/rig_calibrator/bin/rig_utils.py:201-244.

RUNS IN THE BUILD CONTAINER ONLY (the reference never travels): the datasets
and CLI runs are those of make_rig_config_golden.py (zero passes: read,
bracket, write) plus a --no_rig case; the reference reader parses the
CLI-written cameras.txt once per sensor (it keeps the images whose parent
directory is that sensor). Stored per case: the CLI-written text with the
temporary data directory replaced by ``{DATA}``, and per sensor the parsed
image names (same placeholder) and 4x4 world_to_cam matrices.
tests/test_cameras_ref.py re-runs the CLI and checks bytes and values.

    python tests/golden/make_cameras_golden.py
"""
import importlib.util
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
REF_UTILS = "/root/reference/rig_calibrator/bin/rig_utils.py"
OUT = os.path.join(HERE, "cameras_ref_parse.json")

from make_rig_config_golden import CASES as RIG_CASES, CLI, make_case  # noqa: E402

CASES = dict(RIG_CASES)
CASES["radtan_fov_none_no_rig"] = dict(rig=dict(models=["radtan", "fov", "none"], seed=3), args=["--no_rig"])


def load_reader():
    spec = importlib.util.spec_from_file_location("ref_rig_utils", REF_UTILS)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.parse_images_and_camera_poses


def main():
    parse = load_reader()
    subprocess.run(["make", "-s", "-C", os.path.dirname(CLI)], check=True)
    fixtures = {}
    for name, case in CASES.items():
        with tempfile.TemporaryDirectory() as tmp:
            _, written = make_case(case, tmp)
            cams = os.path.join(os.path.dirname(written), "cameras.txt")
            data = os.path.join(tmp, "data")
            sensors = {}
            for s in _sensor_names(case):
                images, w2c = parse(cams, s)
                sensors[s] = {"images": [i.replace(data, "{DATA}") for i in images],
                              "world_to_cam": [m.tolist() for m in w2c]}
            fixtures[name] = {"case": case, "written_text": open(cams).read().replace(data, "{DATA}"),
                              "parsed": sensors}
        print(name, {s: len(v["images"]) for s, v in sensors.items()})
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_cameras_golden.py",
                   "parser": "rig_calibrator/bin/rig_utils.py:201-244 (parse_images_and_camera_poses)",
                   "cases": fixtures}, f, indent=1)
    print("wrote", OUT)


def _sensor_names(case):
    from multiview_amd import rig

    kw = dict(num_ref=8, num_points=150, obs_per_point=4)
    kw.update(case["rig"])
    return list(rig.make_rig(num_sensors=len(kw["models"]), **kw).sensor_names)


if __name__ == "__main__":
    main()
