"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer
(tests/sanitize/Makefile: libmvba's host side, the CLI and the Ceres adapter
built with ROCm clang, -fsanitize=address,undefined on the host compilation
only; GPU code is never sanitized here).

CPU: mvba_create's validation paths and the CLI file formats
(tests/sanitize/san_validate.cpp), the CLI's flag parsing and parameter
validation (rig_calibrator.cc:893-955 messages). GPU: the same driver through a
real handle (host hand-over, depth, deterministic solve), the Ceres adapter
driver (tests/cpp/test_ceres_surface.cpp) and an end-to-end CLI run whose
outputs must equal the plain build's. Any sanitizer report fails the test."""
import os
import subprocess

import pytest

from conftest import ROOT

SAN = os.path.join(ROOT, "tests", "sanitize")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:protect_shadow_gap=0:abort_on_error=0:exitcode=23",
           UBSAN_OPTIONS="print_stacktrace=1")
REPORTS = ("ERROR: AddressSanitizer", "runtime error:", "ERROR: LeakSanitizer")


def _bin(name):
    path = os.path.join(SAN, name)
    if not os.path.exists(path):
        subprocess.run(["make", "-s", "-j8", "-C", SAN, name], check=True)
    return path


def _clean(text):
    bad = [r for r in REPORTS if r in text]
    assert not bad, text[-6000:]


def _run(args, cwd=None, timeout=300):
    p = subprocess.run(args, capture_output=True, text=True, env=ENV, cwd=cwd, timeout=timeout)
    _clean(p.stdout + p.stderr)
    return p


def test_validation_and_formats_under_sanitizers(tmp_path):
    p = _run([_bin("san_validate"), str(tmp_path / "formats")])
    assert p.returncode == 0 and "0 failure(s)" in p.stdout, p.stdout + p.stderr


@pytest.mark.parametrize("extra,msg", [
    (["--robust_threshold=0"], "The robust threshold must be positive."),
    (["--bracket_len", "-1"], "Bracket length must be positive."),
    (["--no_rig", "--float_timestamp_offsets"], "Cannot float timestamps with option --no_rig."),
    (["--camera_poses=x.txt"], "Cannot specify both --nvm and --camera_poses."),
    (["--no_such_flag=3"], "unknown command line flag"),
])
def test_cli_flags_under_sanitizers(tmp_path, extra, msg):
    p = _run([_bin("rig_calibrator_san"), "--rig_config", "r.txt", "--nvm", "c.nvm", "--out_dir", str(tmp_path),
              *extra])
    assert p.returncode == 1 and msg in p.stderr, p.stderr


def test_batch_chain_under_sanitizers():
    """Ceres-adapter batches destroyed out of construction order: no dangling
    'current batch' link (tests/cpp/test_ceres_surface.cpp --chain; no GPU)."""
    p = _run([_bin("test_ceres_surface_san"), "--chain"])
    assert p.returncode == 0 and "chain ok" in p.stdout, p.stdout + p.stderr


@pytest.mark.gpu
def test_device_paths_under_sanitizers(tmp_path, oracle):
    p = _run([_bin("san_validate"), str(tmp_path / "formats")])
    assert p.returncode == 0 and "0 failure(s)" in p.stdout and "ok solve" in p.stdout, p.stdout + p.stderr
    from test_ceres_surface_gpu import run_adapter_case

    _clean(run_adapter_case(_bin("test_ceres_surface_san"), tmp_path, oracle, env=ENV))


@pytest.mark.gpu
def test_cli_end_to_end_under_sanitizers(tmp_path):
    from test_cli import _dataset

    _, info = _dataset(tmp_path, models=("radtan", "rpc1", "fov"))
    outs = {}
    for name, exe in (("plain", os.path.join(ROOT, "multiview_amd", "cli", "rig_calibrator")),
                      ("san", _bin("rig_calibrator_san"))):
        out_dir = tmp_path / name
        p = _run([exe, "--rig_config", info["rig_config"], "--nvm", info["nvm"], "--out_dir", str(out_dir),
                  "--num_iterations", "20", "--intrinsics_to_float", "ref_cam:focal_length cam1:focal_length,distortion", "--save_nvm"])
        assert p.returncode == 0, p.stderr[-3000:]
        outs[name] = {f: open(out_dir / f).read() for f in ("cameras.txt", "rig_config.txt", "cameras.nvm")}
    # same library code, same inputs: the sanitized build must write the same
    # files up to the last printed digits (atomics make the solve order-dependent)
    import numpy as np

    for f in ("cameras.txt",):
        a = [float(x) for x in outs["plain"][f].split() if _isnum(x)]
        b = [float(x) for x in outs["san"][f].split() if _isnum(x)]
        assert len(a) == len(b) and np.allclose(a, b, rtol=1e-6, atol=1e-8)


def _isnum(x):
    try:
        float(x)
        return True
    except ValueError:
        return False
