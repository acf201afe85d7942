"""Does the c3 evaluation's time follow where its output planes land in HBM?
(the same k_eval_local<rpc2> measured 1.82 ms on one box
and 2.19 ms on another with equal copy rates.) In ONE process on one box the
c3 residual + Jacobian planes (11.6 GB) are allocated behind pads of 0 .. 7 x
768 MB (each pad moves the planes to other physical pages / channels), and the
one-launch evaluation is timed with HIP events on its stream, 20 launches per
placement, plus a 1 GiB device copy for the box's copy rate. If the spread
within one box matches the spread across boxes, the placement, not the box,
sets c3's store rate. usage: c3_alloc_probe.py [npads]"""
import json
import os
import subprocess
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from multiview_amd import rig  # noqa: E402
from multiview_amd.evaluator import Evaluator  # noqa: E402

npads = int(sys.argv[1]) if len(sys.argv) > 1 else 8
torch.cuda.set_device(0)
R = rig.make_rig(**rig.CONFIGS["c3"])
P = rig.build_problem(R)
stream = torch.cuda.Stream()
sh = stream.cuda_stream
out = {"config": "c3", "pads_mb": [], "kernel_ms": [], "copy_gbs": []}
try:
    smi = subprocess.run(["rocm-smi", "--showclocks", "--showmemuse", "--showtemp", "--showpower"],
                         capture_output=True, text=True, timeout=30).stdout
except Exception as e:  # noqa: BLE001
    smi = f"rocm-smi unavailable: {e}"
out["smi_before"] = smi
with Evaluator(P, device=0) as ev:
    ev.set_params()
    ld = ev.ld
    with torch.cuda.stream(stream):
        for k in range(npads):
            pad = torch.empty(k * 768 * (1 << 20) // 8 + 1, dtype=torch.float64, device="cuda")
            res = torch.empty((2, ld), dtype=torch.float64, device="cuda")
            jac = torch.empty((ev.stride, ld), dtype=torch.float64, device="cuda")
            for _ in range(3):
                ev.evaluate_device(True, residuals=res, jac=jac, ld=ld, stream=sh)
            torch.cuda.synchronize()
            e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            e[0].record(stream)
            for _ in range(20):
                ev.evaluate_device(True, residuals=res, jac=jac, ld=ld, stream=sh)
            e[1].record(stream)
            torch.cuda.synchronize()
            ev.sync(sh)
            ms = e[0].elapsed_time(e[1]) / 20
            a = torch.empty(1 << 27, dtype=torch.float64, device="cuda")
            b = torch.empty_like(a)
            b.copy_(a)
            torch.cuda.synchronize()
            c = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            c[0].record(stream)
            for _ in range(10):
                b.copy_(a)
            c[1].record(stream)
            torch.cuda.synchronize()
            gbs = 2.0 * a.numel() * 8 / (c[0].elapsed_time(c[1]) / 10 * 1e-3) / 1e9
            out["pads_mb"].append(k * 768)
            out["kernel_ms"].append(ms)
            out["copy_gbs"].append(gbs)
            print(f"pad {k * 768:5d} MB: c3 evaluation {ms:.3f} ms ({ev.num_residuals / (ms * 1e-3):.3e} evals/s), "
                  f"copy {gbs:.0f} GB/s, planes at {jac.data_ptr():#x}", flush=True)
            del pad, res, jac, a, b
            torch.cuda.empty_cache()
k = np.array(out["kernel_ms"])
out["spread"] = {"min_ms": float(k.min()), "max_ms": float(k.max()), "max_over_min": float(k.max() / k.min())}
print(json.dumps(out["spread"]))
os.makedirs("gpurun_out", exist_ok=True)
json.dump(out, open("gpurun_out/c3_alloc_probe.json", "w"), indent=1)
