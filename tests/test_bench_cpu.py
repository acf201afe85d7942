"""bench.py's host-side pieces that need no GPU: the CPU baseline leg (oracle
modes NUMDIFF_FAITHFUL / NUMDIFF / ANALYTIC on a bounded sample, median of
passes) and the BA roofline's algorithmic byte model (DESIGN.md §5 "BA
roofline")."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from multiview_amd import rig  # noqa: E402


def test_cpu_baseline_reports_faithful_lean_and_analytic(oracle):
    R = rig.make_rig(num_sensors=3, num_ref=12, num_points=200, obs_per_point=4, models=["radtan"] * 3, seed=9)
    P = rig.build_problem(R)
    cb = bench.cpu_baseline(P, 400)
    assert cb["kind"] == "port" and cb["unit"] == "evals/s"
    for k in ("value", "lean_value", "analytic_value", "value_16_threads", "value_nproc_threads"):
        assert cb[k] > 0.0, k
    assert cb["cores"] in (bench.CPU_THREADS, cb["usable_cores"], cb["nproc"])
    assert "median of 5 passes" in cb["sample"] and "NUMDIFF_FAITHFUL" in cb["sample"]


def test_cg_bytes_model():
    # c2: 999,605 observations, 100k points, 2,998 frames, 7,040 camera entries, radtan
    b = bench.cg_bytes(999605, 100000, 2998, 7040, [5, 5, 5])
    assert b == 136 * 999605 + 152 * 100000 + 8 * (144 + 132 + 23 + 4 * 14) * 2998 + 704 * 7040
    assert 164e6 < b < 166e6
    # RPC: only the distortion half is live in the direction records
    b_rpc = bench.cg_bytes(10, 1, 1, 1, [44])
    assert b_rpc == 136 * 10 + 152 + 8 * (144 + 132 + 18 + 44 + 4 * (9 + 22)) + 704


@pytest.mark.parametrize("n", [0, 1])
def test_cg_bytes_small(n):
    assert bench.cg_bytes(n, n, n, n, []) == (136 + 152 + 8 * (276 + 18 + 36) + 704) * n


def test_committed_summaries_apply_to_whole_config_only():
    # profiles/ PMC summaries are per launch of the whole config on one GPU
    assert bench.summaries_apply(1, 1)
    assert not bench.summaries_apply(1, 8)   # --shard-of rehearsal
    assert not bench.summaries_apply(2, 1)   # an N > 1 rank
    assert not bench.summaries_apply(8, 1)
