"""bench.py --gpus N: the launcher logic (no GPU needed).

`python bench.py --gpus N` must measure N ranks however it is started: under a
launcher (WORLD_SIZE set) it is one rank; without one it starts the N ranks
itself (torch.distributed.run as a child) or refuses an impossible request."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def plan(gpus, env=None, ndev=8, backend="nccl"):
    return bench.launch_plan(gpus, env or {}, ndev, backend, "/x/bench.py", ["--gpus", str(gpus)], 29500)


def test_single_gpu_runs_in_process():
    assert plan(1) is None


def test_under_a_launcher_is_a_rank():
    assert plan(4, env={"WORLD_SIZE": "4"}) is None


def test_launcher_world_mismatch_refused():
    with pytest.raises(SystemExit, match="WORLD_SIZE 2"):
        plan(4, env={"WORLD_SIZE": "2"})


def test_spawns_n_ranks_without_launcher():
    cmd = plan(8)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=8" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29500"
    assert cmd[-3:] == ["/x/bench.py", "--gpus", "8"]


def test_more_ranks_than_gpus_refused_for_rccl():
    with pytest.raises(SystemExit, match="only 8 GPU"):
        plan(9, ndev=8)


def test_gloo_rehearsal_may_share_a_gpu():
    cmd = plan(2, ndev=1, backend="gloo")
    assert "--nproc-per-node=2" in cmd


def test_no_gpu_refused():
    with pytest.raises(SystemExit, match="no GPU"):
        plan(2, ndev=0, backend="gloo")
    with pytest.raises(SystemExit, match="at least one"):
        plan(0)


def test_cli_exits_nonzero_without_gpus():
    """The parent refuses before any rank starts (this container has no GPU)."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode != 0
    assert "no GPU visible" in p.stderr


def test_kernel_degree_names():
    assert bench.kernel_degree("radtan") == "2, 0"
    assert bench.kernel_degree("rpc2") == "3, 2"
    assert bench.kernel_degree("none") == "0, 0"
