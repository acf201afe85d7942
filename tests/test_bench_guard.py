"""bench.py's failure path for its later phases (no GPU needed).

The driver's first N > 1 run is the first time RCCL runs at world > 1, so a
failure there must not cost the evaluation headline: PhaseGuard records an
exception from any rank in the line under the phase's key, every rank skips the
phases after it, and bench.py exits non-zero after printing the line. With two
gloo ranks on the CPU the ranks agree on the failure over the control group."""
import json
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _boom():
    raise RuntimeError("exchange failed")


def test_single_rank_failure_recorded_and_later_phases_skipped():
    line = {"value": 1.0e10, "linearize": None}
    g = bench.PhaseGuard(line, 1, 0)
    assert g.run("linearize", lambda: line.__setitem__("linearize", {"kernel_ms": 0.07}))
    assert not g.run("ba", _boom)
    assert not g.run("weak", lambda: line.__setitem__("weak", {"value": 1.0}))
    assert line["value"] == 1.0e10 and line["linearize"] == {"kernel_ms": 0.07}
    assert line["ba"]["error"] == "rank 0: RuntimeError: exchange failed"
    assert line["weak"] == {"skipped": "an earlier phase failed on some rank"}
    assert line["errors"] == {"ba": ["rank 0: RuntimeError: exchange failed"]}
    json.dumps(line)  # still one printable JSON line


def test_injection_spec():
    assert bench.injected_failure("exchange@1", 1)
    assert not bench.injected_failure("exchange@1", 0)
    assert not bench.injected_failure("", 1)
    assert not bench.injected_failure("exchange", 1)
    with pytest.raises(RuntimeError, match="injected"):
        bench.FailingExchange(None)(0, 1, 0, 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctrl = dist.new_group(backend="gloo")
    line = {"value": 2.0e10}
    g = bench.PhaseGuard(line, world, rank, ctrl)
    g.run("linearize", lambda: None)
    g.run("ba", _boom if rank == 1 else (lambda: None))
    g.run("weak", lambda: line.__setitem__("weak", {"value": 1.0}))
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(line, f)
    dist.barrier(group=ctrl)
    dist.destroy_process_group()


def test_two_ranks_agree_on_a_failure(tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        line = json.load(open(tmp_path / f"rank{r}.json"))
        assert line["value"] == 2.0e10
        assert "linearize" not in line or "error" not in line.get("linearize", {})
        assert line["ba"]["error"] == "rank 1: RuntimeError: exchange failed", line
        assert line["weak"] == {"skipped": "an earlier phase failed on some rank"}
