"""bench.py --gpus 2 with an injected exchange failure (gloo rehearsal, both
ranks on one GPU): the LM phase of rank 1 fails at its first exchange, rank 0's
matching exchange times out (--dist-timeout), the line still prints with the
evaluation headline and `ba.error`, and the run exits non-zero."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_injected_exchange_failure_keeps_the_headline():
    env = dict(os.environ, MVBA_BENCH_INJECT="exchange@1", HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--config", "c2",
           "--steps", "20", "--warmup", "2", "--ba-iters", "2", "--dist-timeout", "20", "--no-cpu-baseline",
           "--mesh-subdiv", "0"]
    p = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=240, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    out_dir = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out_dir):  # the whole run for inspection (pytest truncates messages)
        with open(os.path.join(out_dir, "bench_failure_test.log"), "w") as f:
            f.write(p.stdout + "\n---- stderr\n" + p.stderr)
    assert p.returncode != 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert len(lines) == 1, p.stdout[-2000:] + p.stderr[-4000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert "injected exchange failure" in line["ba"].get("error", ""), line.get("errors")
    assert line["weak"]["skipped"]
