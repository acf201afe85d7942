#!/usr/bin/env python3
"""Where a k_eval_local wave spends its time: run rank 0's shard of an N-way
split of a config (default c2, N = 8) through a -DMVBA_EVAL_STAMPS build
(tools/build_variant.sh stamps -DMVBA_EVAL_STAMPS; loaded through MVBA_LIB),
evaluate a few times, read the per-wave real-time stamps (100 MHz) of the
last launch and print the phase durations: entry -> segment record -> frame
descriptor and a parameter through it -> K0's common part -> K0's pose
columns -> projection done (landmark
/ measurement loads consumed) -> every store issued -> every store
acknowledged; plus the spread of wave start and end times over the launch.

usage: MVBA_LIB=tools/ab/stamps/libmvba.so python3 tools/eval_stamps.py [--config c2] [--shard-of 8]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--shard-of", type=int, default=8)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch

    from multiview_amd import rig
    from multiview_amd.evaluator import Evaluator

    cfg = dict(rig.CONFIGS[a.config])
    R = rig.make_rig(**cfg)
    if a.shard_of > 1:
        R = rig.shard_points(R, 0, a.shard_of)
    P = rig.build_problem(R, rig.FloatFlags(**rig.CONFIG_FLAGS.get(a.config, {})))
    ev = Evaluator(P, device=0)
    ev.set_params()
    ld = ev.ld
    res = torch.empty((2, ld), dtype=torch.float64, device="cuda")
    jac = torch.empty((ev.stride, ld), dtype=torch.float64, device="cuda")
    for _ in range(20):
        ev.evaluate_device(True, residuals=res, jac=jac, ld=ld)
    torch.cuda.synchronize()
    ev.sync(0)
    nst = 8
    nw = 16384
    buf = (C.c_ulonglong * (nw * nst))()
    ev.lib.mvba_debug_eval_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    rc = ev.lib.mvba_debug_eval_stamps(buf, nw * nst)
    assert rc == 0, rc
    t = np.frombuffer(buf, dtype=np.uint64).reshape(nw, nst).astype(np.int64)
    nseg = int((t[:, 0] > 0).sum())
    t = t[:nseg]
    follower = t[:, 7] == 0  # (MVBA_K0_SHARE) waves that took the record of their block's first wave of the frame
    t[follower, 7] = t[follower, 6]
    ok = (t > 0).all(axis=1)
    t = t[ok]
    us = 0.01  # 100 MHz ticks
    # columns: 0 entry, 5 segment record, 6 frame descriptor + a parameter,
    # 7 K0's common part done (lane 0), 1 K0 done, 2 projection done,
    # 3 stores issued, 4 stores acknowledged
    t = t[:, [0, 5, 6, 7, 1, 2, 3, 4]]
    d = np.diff(t, axis=1) * us
    names = ["segment record load", "frame descriptor + parameter loads", "K0 common part",
             "K0 pose columns + barrier", "loads + projection", "stores issued", "stores acknowledged"]
    out = {"config": a.config, "shard_of": a.shard_of, "waves": int(len(t)), "form": ev.eval_form(),
           "k0_waves": int((~follower[ok]).sum()),
           "launch_span_us": float((t[:, -1].max() - t[:, 0].min()) * us),
           "wave_start_spread_us": float((t[:, 0].max() - t[:, 0].min()) * us),
           "wave_life_us": {"median": float(np.median((t[:, -1] - t[:, 0]) * us)),
                            "p90": float(np.percentile((t[:, -1] - t[:, 0]) * us, 90)),
                            "max": float(((t[:, -1] - t[:, 0]) * us).max())},
           "phases_us": {n: {"median": float(np.median(d[:, k])), "p90": float(np.percentile(d[:, k], 90))}
                         for k, n in enumerate(names)}}
    print(json.dumps(out, indent=1))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)
    ev.close()


if __name__ == "__main__":
    main()
