#!/usr/bin/env python3
"""Where the evaluation step's non-kernel time goes (timing tool, one GPU).

For rank 0's shard of an N-way landmark split of c2 (N = 1, 8), time K
evaluation steps three ways: (a) the bench loop (two library calls per step
with three HIP events between them), (b) one library call per step and no
events, (c) the K steps captured once in a HIP graph (torch.cuda.graph over
the library's launches on the capturing stream) and replayed once.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from multiview_amd import _lib, rig
    from multiview_amd.evaluator import Evaluator

    K = 200
    for split in (1, 8):
        cfg = dict(rig.CONFIGS["c2"])
        n = cfg["num_points"]
        cfg["point_range"] = (0, n // split)
        P = rig.build_problem(rig.make_rig(**cfg), rig.FloatFlags(**rig.CONFIG_FLAGS.get("c2", {})))
        ev = Evaluator(P, device=0)
        ev.set_params()
        res = torch.empty((2, ev.ld), dtype=torch.float64, device="cuda")
        jac = torch.empty((ev.stride, ev.ld), dtype=torch.float64, device="cuda")
        side = torch.cuda.Stream()
        out = {}
        with torch.cuda.stream(side):
            sh = side.cuda_stream
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(3 * K)]

            def run(mode):
                for k in range(K):
                    if mode == "a":
                        evs[3 * k].record(side)
                        ev.evaluate_device(True, residuals=res, jac=jac, ld=ev.ld, stream=sh,
                                           phase=_lib.EVAL_PREP_ONLY)
                        evs[3 * k + 1].record(side)
                        ev.evaluate_device(True, residuals=res, jac=jac, ld=ev.ld, stream=sh,
                                           phase=_lib.EVAL_SKIP_PREP)
                        evs[3 * k + 2].record(side)
                    else:
                        ev.evaluate_device(True, residuals=res, jac=jac, ld=ev.ld, stream=sh)

            for mode in ("a", "b"):
                run(mode)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                run(mode)
                torch.cuda.synchronize()
                out[mode] = (time.perf_counter() - t0) / K * 1e6
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=side):
                sh = side.cuda_stream
                run("b")
            g.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            out["c"] = (time.perf_counter() - t0) / K * 1e6
        ev.sync()
        print(f"1/{split} shard ({ev.num_residuals} obs): us per step  (a) bench loop {out['a']:.1f}  "
              f"(b) one call, no events {out['b']:.1f}  (c) hipGraph of {K} steps {out['c']:.1f}", flush=True)
        ev.close()


if __name__ == "__main__":
    main()
