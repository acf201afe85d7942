"""Run the Ceres-surface hand-over (mvba_evaluate_packed into pinned memory) at
c2 a few times: a short program for rocprofv3 --pmc passes over k_rows."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from multiview_amd import rig  # noqa: E402
from multiview_amd.evaluator import Evaluator, PinnedBuffer  # noqa: E402

cfg = dict(rig.CONFIGS["c2"])
R = rig.make_rig(**cfg)
P = rig.build_problem(R, rig.FloatFlags(**rig.CONFIG_FLAGS.get("c2", {})))
with Evaluator(P) as ev:
    ev.set_params()
    off = ev.set_transfer_blocks(None)
    with PinnedBuffer(int(off[-1])) as buf, PinnedBuffer(2 * ev.num_residuals) as rb:
        for k in range(6):
            t = time.perf_counter()
            ev.evaluate_packed(jacobian=True, apply_loss=True, out=buf.array, res_out=rb.array, want_cost=False)
            print(f"packed evaluation {k}: {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
