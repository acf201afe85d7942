"""Run the sanitized rig_calibrator on tests/test_sanitize.py's CLI case and
keep the whole stderr (gpurun_out/san_cli_<tag>.log), for reading an ASan
report the test truncates. usage: san_cli_repro.py TAG [ENV=VAL ...]"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from pathlib import Path  # noqa: E402

from test_cli import _dataset  # noqa: E402

tag = sys.argv[1]
env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:protect_shadow_gap=0:abort_on_error=0:exitcode=23",
           UBSAN_OPTIONS="print_stacktrace=1")
for kv in sys.argv[2:]:
    k, v = kv.split("=", 1)
    env[k] = v
with tempfile.TemporaryDirectory() as td:
    _, info = _dataset(Path(td), models=("radtan", "rpc1", "fov"))
    exe = os.path.join(ROOT, "tests", "sanitize", "rig_calibrator_san")
    p = subprocess.run([exe, "--rig_config", info["rig_config"], "--nvm", info["nvm"], "--out_dir",
                        os.path.join(td, "out"), "--num_iterations", "20", "--intrinsics_to_float",
                        "ref_cam:focal_length cam1:focal_length,distortion", "--save_nvm"],
                       capture_output=True, text=True, env=env, timeout=300)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", f"san_cli_{tag}.log"), "w") as f:
    f.write(f"rc {p.returncode}\n--- stdout\n{p.stdout}\n--- stderr\n{p.stderr}")
print(tag, "rc", p.returncode)
