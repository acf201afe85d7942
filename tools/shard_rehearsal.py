#!/usr/bin/env python3
"""Rehearsal of the device-resident sharded solve on ONE GPU.

c2 (or --config) split into --shards landmark ranges, one thread + HIP stream
per shard, all on cuda:0, exchanging through the library's local communicator
(mvba_comm_init_local: stream-ordered device all-reduce, no host staging; RCCL
refuses two ranks on one device). Prints one JSON line: the unsharded solve
and the sharded one (LM iterations, CG iterations, ms per CG iteration), so the
per-CG-iteration exchange cost is the difference at equal work per iteration
(on one GPU the shards' kernels share the device: the sharded time is the
unsharded time plus the exchange, not divided by the shard count).

    python tools/shard_rehearsal.py --config c2 --shards 2 --iters 5
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--shards", type=int, default=2)
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    import torch

    from multiview_amd import rig
    from multiview_amd.dist import Comm, shard_range
    from multiview_amd.evaluator import Evaluator

    torch.cuda.set_device(0)
    cfg = dict(rig.CONFIGS[args.config])
    flags = rig.FloatFlags(**rig.CONFIG_FLAGS.get(args.config, {}))
    kw = dict(max_num_iterations=args.iters, function_tolerance=0.0, gradient_tolerance=0.0,
              parameter_tolerance=0.0, use_loss=1, robust_threshold=3.0)
    out = {"config": args.config, "shards": args.shards}

    # unsharded
    P = rig.build_problem(rig.make_rig(**cfg), flags)
    st = torch.cuda.Stream()
    with Evaluator(P) as ev:
        ev.set_params()
        ev.solve(**dict(kw, max_num_iterations=1), stream=st.cuda_stream)
        ev.set_params()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s = ev.solve(**kw, stream=st.cuda_stream)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    out["unsharded"] = dict(wall_s=dt, lm=s["num_iterations"], cg=s["num_linear_iterations"],
                            ms_per_cg=1e3 * s["linear_solver_time_s"] / max(s["num_linear_iterations"], 1),
                            final_cost=s["final_cost"])
    del P

    # sharded, one process
    n = args.shards
    comms = Comm.local([0] * n)
    evs = []
    for r in range(n):
        c = dict(cfg, point_range=shard_range(cfg["num_points"], n, r))
        Pr = rig.build_problem(rig.make_rig(**c), flags)
        ev = Evaluator(Pr, device=0)
        evs.append(ev)
    streams = [torch.cuda.Stream() for _ in range(n)]
    res = [None] * n

    def run(r, k):
        try:
            res[r] = evs[r].solve(**dict(kw, max_num_iterations=k), comm=comms[r], stream=streams[r].cuda_stream)
        except Exception as e:  # noqa: BLE001
            res[r] = e
            comms[r].abort()

    for k in (1, args.iters):  # warm-up, then timed
        for ev in evs:
            ev.set_params()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        th = [threading.Thread(target=run, args=(r, k)) for r in range(n)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    bad = [x for x in res if isinstance(x, Exception)]
    if bad:
        raise bad[0]
    s = res[0]
    out["sharded"] = dict(wall_s=dt, lm=s["num_iterations"], cg=s["num_linear_iterations"],
                          ms_per_cg=1e3 * s["linear_solver_time_s"] / max(s["num_linear_iterations"], 1),
                          final_cost=s["final_cost"],
                          same_cost_all_shards=all(x["final_cost"] == s["final_cost"] for x in res))
    out["exchange_us_per_cg_iteration"] = 1e3 * (out["sharded"]["ms_per_cg"] - out["unsharded"]["ms_per_cg"])
    print(json.dumps(out), flush=True)
    for ev in evs:
        ev.close()
    for c in comms:
        c.close()


if __name__ == "__main__":
    main()
