#!/usr/bin/env python3
"""Fixtures that pin the CLI's rig_config.txt writer (writeRigConfig,
dense_map_utils.cc:779-850) against the reference's own Python parser,
``parseRigConfig`` in /root/reference/rig_calibrator/bin/rig_utils.py:84-185.

RUNS IN THE BUILD CONTAINER ONLY (the reference never travels): for each case a
synthetic dataset is written (multiview_amd.rig_files), the rig_calibrator CLI
runs with --calibrator_num_passes 0 (CPU only: read config + NVM, bracket, write
outputs), and the reference parser reads both the input configuration and the
CLI-written one. Stored per case: the generator arguments, the CLI arguments,
the CLI-written text, and both parses (lists of per-sensor dicts of strings, as
parseRigConfig returns them). tests/test_rig_config_ref.py re-runs the CLI on
the regenerated dataset and checks the text byte for byte and the parsed values.

parseRigConfig accepts 0, 1, 4 or 5 distortion coefficients only (rig_utils.py:141),
so RPC sensors are not among the cases.

    python tests/golden/make_rig_config_golden.py
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
REF_UTILS = "/root/reference/rig_calibrator/bin/rig_utils.py"
CLI = os.path.join(ROOT, "multiview_amd", "cli", "rig_calibrator")
OUT = os.path.join(HERE, "rig_config_ref_parse.json")

CASES = {
    "radtan_fov_none_initial_rig": dict(rig=dict(models=["radtan", "fov", "none"], seed=3),
                                         args=["--use_initial_rig_transforms"]),
    "radtan_fov_none_rig_from_poses": dict(rig=dict(models=["radtan", "fov", "none"], seed=3), args=[]),
    "radtan4_radtan_initial_rig": dict(rig=dict(models=["radtan4", "radtan", "none", "fov"], seed=11),
                                       args=["--use_initial_rig_transforms"]),
    "depth_sensor_initial_rig": dict(rig=dict(models=["radtan", "fov", "none"], seed=5, depth_sensors=(2,)),
                                     args=["--use_initial_rig_transforms"], depth=True),
}


def load_parser():
    spec = importlib.util.spec_from_file_location("ref_rig_utils", REF_UTILS)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.parseRigConfig


def make_case(case, tmp):
    """Shared with the test: dataset + CLI run, returns (input path, written path)."""
    import numpy as np

    from multiview_amd import rig, rig_files

    kw = dict(num_ref=8, num_points=150, obs_per_point=4)
    kw.update(case["rig"])
    models = kw["models"]
    R = rig.make_rig(num_sensors=len(models), **kw)
    dti = None
    if case.get("depth"):
        dti = np.tile(np.eye(4), (len(models), 1, 1))
        for s in range(len(models)):
            a = R.init["depth_to_image"][s]
            dti[s, :3, :3] = rig.quat_to_mat(a[3:][None])[0]
            dti[s, :3, 3] = a[:3]
    info = rig_files.write_dataset(R, os.path.join(tmp, "data"), depth_to_image=dti)
    out = os.path.join(tmp, "out")
    p = subprocess.run([CLI, "--rig_config", info["rig_config"], "--nvm", info["nvm"], "--out_dir", out,
                        "--calibrator_num_passes", "0", *case["args"]], capture_output=True, text=True, timeout=300)
    if p.returncode != 0:
        raise RuntimeError(p.stderr)
    return info["rig_config"], os.path.join(out, "rig_config.txt")


def main():
    parse = load_parser()
    subprocess.run(["make", "-s", "-C", os.path.dirname(CLI)], check=True)
    fixtures = {}
    for name, case in CASES.items():
        with tempfile.TemporaryDirectory() as tmp:
            inp, written = make_case(case, tmp)
            fixtures[name] = {
                "case": case,
                "written_text": open(written).read(),
                "parsed_written": parse(written),
                "parsed_input": parse(inp),
            }
        print(name, len(fixtures[name]["parsed_written"]), "sensors")
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_rig_config_golden.py",
                   "parser": "rig_calibrator/bin/rig_utils.py:84-185 (parseRigConfig)",
                   "cases": fixtures}, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
