"""Generate a synthetic rig_calibrator dataset of a bench configuration and run
the CLI on it (end-to-end wall time, per-phase timings with --profile).

    python tools/cli_run.py --config c2 --out gpurun_out/cli_c2 [-- extra CLI flags]
"""
import argparse
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from multiview_amd import rig, rig_files  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "cli_run"))
    ap.add_argument("extra", nargs="*")
    a = ap.parse_args()
    t = time.time()
    cfg = dict(rig.CONFIGS[a.config])
    R = rig.make_rig(**cfg)
    data = os.path.join(a.out, "data")
    info = rig_files.write_dataset(R, data)
    print(f"dataset {a.config}: {len(R.cam_type)} images, {R.xyz.shape[0]} points, {R.obs_pid.size} features, "
          f"written in {time.time() - t:.1f} s", flush=True)
    cli = os.path.join(ROOT, "multiview_amd", "cli", "rig_calibrator")
    cmd = [cli, "--rig_config", info["rig_config"], "--nvm", info["nvm"], "--out_dir", os.path.join(a.out, "out"),
           "--profile"] + a.extra
    t = time.time()
    with open(os.path.join(a.out, "cli.log"), "w") as f:
        p = subprocess.run(cmd, stdout=f, stderr=subprocess.STDOUT)
    print(f"rig_calibrator exit {p.returncode}, wall {time.time() - t:.2f} s", flush=True)
    # drop the bulky inputs, keep the log and the outputs
    import shutil

    shutil.rmtree(data, ignore_errors=True)
    sys.exit(p.returncode)


if __name__ == "__main__":
    main()
