#!/usr/bin/env python3
"""Benchmark of the rig_calibrator evaluator hot path on MI355X.

Metric (BASELINE.json): residual+Jacobian evals/sec, 3-cam rig, 1M obs.
Workload (configs[1], "c2"): 3-sensor rig, 100k landmarks / 1M observations,
radial-tangential distortion (K=5), fp64, every block floating. A STEP is one
full pass of the hot path over all observations with inputs resident in HBM:
point gather + per-frame pose kernel (K0) + per-observation residual and
analytic Jacobian kernel (K1), outputs written to HBM (materialised Ceres
columns).

Multi-GPU (one process per GPU, torchrun): observations are sharded by
landmark range. The headline is STRONG scaling: the config's
landmarks (c2: 100k landmarks / 1M observations) are the whole job, split into
N contiguous landmark ranges of capture order (rig.shard_points: landmarks by
the timestamp of their first observing image, equal observation counts);
evaluation has no data-path collective; value =
all ranks' evals / max time. With N > 1 a "weak" object adds the weak-scaling
line (each rank owns a config-sized shard of an N x larger problem). The LM
phase exchanges through the library's RCCL communicator (mvba_comm, stream-
ordered ncclAllReduce on the solver's stream).

Also reported: "roofline" of the dominant kernel (K1, radtan) from HIP events on
its launch stream, and "cpu_baseline" = the oracle's restatement of the
reference evaluator (oracle/: the functor with its per-call CameraParameters
copies inside Ceres 1.14 central differences), median of 5 passes after a
warm-up, timed on this host.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP64_PEAK_TFLOPS = 78.6  # MI355X fp64 vector (= fp64 matrix) peak, AMD product specification
CPU_THREADS = 16       # reference default --num_opt_threads (rig_calibrator.cc:256)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ba-iters", type=int, default=5, help="LM iterations timed in phase C (0 = skip)")
    ap.add_argument("--cpu-sample", type=int, default=0, help="residuals in the CPU sample (0 = auto)")
    ap.add_argument("--mesh-subdiv", type=int, default=7,
                    help="icosphere level of the --mesh ray-intersection line (0 = skip; 7 = 327,680 faces)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, default) or gloo (rehearsal of the multi-rank path on one GPU)")
    ap.add_argument("--shard-of", type=int, default=1,
                    help="single-process rehearsal: run rank 0's shard of an N-way strong split (timing only)")
    ap.add_argument("--ba-deadline", type=float, default=120.0,
                    help="N > 1: seconds the LM phase may take before its RCCL communicator is aborted (the "
                         "failure is recorded in the line, which still prints); also the communicator's "
                         "init / enqueue deadline")
    ap.add_argument("--dist-timeout", type=float, default=300.0,
                    help="N > 1: torch.distributed collective timeout (s)")
    ap.add_argument("--ba-exchange", default="auto", choices=("auto", "rccl"),
                    help="auto: the exchange N > 1 takes (RCCL), none at N = 1; rccl: at N = 1 too, through a "
                         "one-rank RCCL communicator (rehearsal of the sharded LM path: fold-mode CG tail, the "
                         "ncclAllReduce inside the captured CG runs), e.g. with --shard-of 8")
    ap.add_argument("--scaling", default="strong", choices=("strong", "weak"),
                    help="strong (default): the config is the whole job, split over the ranks; "
                         "weak: every rank owns a config-sized shard")
    return ap.parse_args()


def launch_plan(gpus, environ, device_count, backend, script, argv, port):
    """How `bench.py --gpus N` runs. Returns None when this process is itself a
    rank (a launcher set WORLD_SIZE, or N == 1), else the command that starts
    the N ranks as a child (torch.distributed.run on 127.0.0.1). Raises
    SystemExit for an impossible request, before anything touches the GPU:
    RCCL needs N distinct devices; the gloo rehearsal may share them."""
    if gpus < 1:
        raise SystemExit(f"--gpus {gpus}: need at least one GPU")
    world = environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != gpus:
            raise SystemExit(f"--gpus {gpus} but the launcher set WORLD_SIZE {world}")
        return None
    if gpus == 1:
        return None
    if device_count < 1:
        raise SystemExit(f"--gpus {gpus}: no GPU visible")
    if backend == "nccl" and device_count < gpus:
        raise SystemExit(f"--gpus {gpus}: only {device_count} GPU(s) visible (RCCL needs one GPU per rank; "
                         f"--dist-backend gloo rehearses the multi-rank path on fewer)")
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), script] + list(argv)


def summaries_apply(world, shard_of):
    """The committed per-launch PMC summaries (profiles/: K1 traffic, fp64
    counts, the CG iteration's kernels) were measured on the whole config on
    one GPU; a line uses them only when it runs exactly that workload."""
    return world == 1 and shard_of <= 1


class PhaseGuard:
    """Runs the bench's later phases (K2 + exchange, the LM solve, the weak-
    scaling line) so that a failure cannot cost the evaluation headline: an
    exception on any rank is recorded in the line under the phase's key
    ({"error": "rank r: ..."}) and in line["errors"], every rank then skips the
    phases that would need the others, and the caller exits non-zero after the
    line is printed. With world > 1 the ranks agree over `ctrl`, a gloo group on
    the CPU (independent of the RCCL communicators' state)."""

    def __init__(self, line, world, rank, ctrl=None):
        self.line, self.world, self.rank, self.ctrl = line, world, rank, ctrl
        self.errors = {}
        self.failed = False

    def run(self, name, fn):
        import torch.distributed as dist

        if self.failed:
            if not isinstance(self.line.get(name), dict):
                self.line[name] = {}
            self.line[name]["skipped"] = "an earlier phase failed on some rank"
            return False
        err = None
        # progress on stderr (long phases at c3 / c4 would otherwise be silent
        # for minutes; stdout carries only the one JSON line)
        print(f"[bench] rank {self.rank}: phase {name}", file=sys.stderr, flush=True)
        try:
            fn()
        except Exception as e:  # noqa: BLE001 - recorded in the line
            err = f"rank {self.rank}: {type(e).__name__}: {e}"
        if self.world > 1:
            errs = [None] * self.world
            dist.all_gather_object(errs, err, group=self.ctrl)
            errs = [e for e in errs if e]
        else:
            errs = [err] if err else []
        if errs:
            self.failed = True
            self.errors[name] = errs
            if not isinstance(self.line.get(name), dict):
                self.line[name] = {}
            self.line[name]["error"] = "; ".join(errs)
            self.line["errors"] = self.errors
        return not errs


def kernel_degree(model):
    """The '<MODEL, DEG' template prefix of the kernels instantiated for a
    rig.py model name (mvba_types.h ModelKind): radtan -> '2, 0', rpc2 -> '3, 2'."""
    if model.startswith("rpc"):
        return f"3, {int(model[3:])}"
    return {"none": "0, 0", "fov": "1, 0", "radtan": "2, 0", "radtan4": "2, 0"}[model]


def injected_failure(spec, rank):
    """Test hook (MVBA_BENCH_INJECT="exchange@R"): rank R's LM-phase exchange
    fails, to rehearse the failure path of an N > 1 run."""
    if not spec:
        return False
    what, _, who = spec.partition("@")
    return what == "exchange" and who.isdigit() and int(who) == rank


class FailingExchange:
    """An exchange callback that fails at its first call (injected failure)."""

    def __init__(self, inner):
        self.inner = inner
        self.calls = 0

    def __call__(self, ptr, count, op, stream=0):
        raise RuntimeError("injected exchange failure (MVBA_BENCH_INJECT)")


def _free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def maybe_launch(args):
    """Start the ranks as a child process when --gpus N > 1 was given without a
    launcher; returns its exit code, or None to run here. torch.cuda.device_count()
    does not initialise the GPU, so no GPU state exists in this parent."""
    import subprocess

    if args.gpus == 1 and "WORLD_SIZE" not in os.environ:
        return None
    import torch

    cmd = launch_plan(args.gpus, os.environ, torch.cuda.device_count(), args.dist_backend,
                      os.path.abspath(__file__), sys.argv[1:], _free_port())
    if cmd is None:
        return None
    env = dict(os.environ)
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    env.setdefault("OMP_NUM_THREADS", "4")
    print(f"bench.py: launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


def _time_numdiff(oracle_py, problem, n, threads, mode, runs=5):
    """BASELINE.md's protocol: one warm-up pass over the first n blocks, then the
    median of `runs` timed passes. Returns (evals/s, [pass seconds])."""
    oracle_py.evaluate_mt(problem, mode, 0, n, threads=threads)  # warm-up
    dts = []
    for _ in range(runs):
        t0 = time.perf_counter()
        oracle_py.evaluate_mt(problem, mode, 0, n, threads=threads)
        dts.append(time.perf_counter() - t0)
    return n / float(np.median(dts)), dts


def _cgroup_cpu_quota():
    """CPUs granted by the cgroup v2 quota (cpu.max 'quota period'), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else max(1, int(-(-int(q) // int(p))))
    except (OSError, ValueError):
        return None


def cpu_baseline(problem, sample: int):
    """The reference's evaluator restated on the CPU, on the first `sample`
    residual blocks (all by default), BASELINE.md's protocol (median of 5 passes
    after 1 warm-up), at the reference's default 16 threads (--num_opt_threads,
    rig_calibrator.cc:256) and at every host core this process may use
    ("all host cores (nproc, stated) and 16 threads").

    `value` is oracle mode NUMDIFF_FAITHFUL: per block the functor with its
    per-call CameraParameters deep copy, heap distortion vector and SetDistortion
    (rig_calibrator.cc:460-467, camera_params.cc:169-208), compute_rpc's
    validation and vectors (rpc_distortion.cc:116-124), and Ceres 1.14's
    DynamicNumericDiffCostFunction / ResidualBlock::Evaluate bookkeeping around
    the central differences (1 + 2*n_free functor calls per block), at the
    faster thread count. `lean_value` is the same numbers without the per-call
    copies (oracle mode NUMDIFF, round 2's baseline); both produce bit-identical
    residuals and Jacobians (tests/test_oracle.py)."""
    from oracle import oracle_py

    n = min(sample, problem.num_residuals) if sample else problem.num_residuals
    oracle_py.load()
    nproc = os.cpu_count() or 1
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    quota = _cgroup_cpu_quota()
    if quota:
        usable = min(usable, quota)
    runs = {}
    for threads in sorted({CPU_THREADS, usable, nproc}):
        runs[threads] = _time_numdiff(oracle_py, problem, n, threads, oracle_py.NUMDIFF_FAITHFUL)
    best = max(runs, key=lambda t: runs[t][0])
    lean = _time_numdiff(oracle_py, problem, n, best, oracle_py.NUMDIFF)
    # the oracle's analytic evaluator on the same sample ("also
    # report the build's analytic CPU evaluator on the same cores")
    ana = _time_numdiff(oracle_py, problem, n, best, oracle_py.ANALYTIC, runs=3)
    return {"value": runs[best][0], "unit": "evals/s", "cores": best, "kind": "port",
            "nproc": nproc, "usable_cores": usable, "cgroup_cpu_quota": quota,
            "value_16_threads": runs[CPU_THREADS][0], "value_nproc_threads": runs[nproc][0],
            "sample": f"median of 5 passes after 1 warm-up over {n} of {problem.num_residuals} residual blocks of "
                      f"the same workload, {best} OpenMP threads (pass times "
                      + ", ".join(f"{t:.2f}" for t in runs[best][1]) + " s): oracle NUMDIFF_FAITHFUL = the "
                      f"reference functor with its per-call CameraParameters copy + SetDistortion, inside Ceres "
                      f"1.14 DynamicNumericDiffCostFunction<CENTRAL> (1 + 2*n_free calls per block); also timed at "
                      + ", ".join(f"{t} threads: {runs[t][0]:.3e} evals/s" for t in sorted(runs))
                      + f" (nproc {nproc}; affinity/cgroup quota leave {usable} cores to this process)",
            "lean_value": lean[0],
            "lean_sample": f"oracle NUMDIFF (same numbers, no per-call copies), median of 5 passes, {best} threads",
            "analytic_value": ana[0],
            "analytic_sample": f"oracle ANALYTIC (exact derivative, dual numbers), median of 3 passes over the same "
                               f"{n} blocks, {best} threads"}


def _stream_copy_gbs(torch, stream, nbytes=1 << 30, reps=10):
    """Device-to-device copy of a 1 GiB buffer (read + write bytes / time) on the
    bench stream, HIP events around `reps` copies: the achievable HBM rate the
    K1 number is also reported against."""
    a = torch.empty(nbytes // 8, dtype=torch.float64, device="cuda").fill_(1.0)
    b = torch.empty_like(a)
    b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        b.copy_(a)
    e1.record(stream)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    del a, b
    return 2.0 * nbytes / (ms * 1e-3) / 1e9


PROFILE_ROUNDS = ("r06", "r05", "r04", "r03", "r02", "r01")  # newest first: committed PMC summaries are read from here


def _profile_path(name):
    here = os.path.dirname(os.path.abspath(__file__))
    for r in PROFILE_ROUNDS:
        path = os.path.join(here, "profiles", r, name)
        if os.path.exists(path):
            return path
    return os.path.join(here, "profiles", PROFILE_ROUNDS[-1], name)


def _pmc_traffic(config, kind="eval"):
    """HBM bytes per launch from the committed PMC summary of this config
    (tools/pmc_summary.py over separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
    passes of this same command; profiles/), or None. kind "eval": the
    one-launch evaluation (k_eval_local / k_eval, pmc_eval_<cfg>.json); "k1":
    the split form's K1 (k_obs, pmc_k1_<cfg>.json); "depth": K1-depth
    (k_depth_obs<double>, pmc_depth_<cfg>.json)."""
    path = _profile_path(f"pmc_{kind}_{config}.json")
    try:
        with open(path) as f:
            return float(json.load(f)["traffic_bytes_per_launch"])
    except (OSError, ValueError, KeyError):
        return None


def _pmc_flops(config):
    """fp64 flops per launch of each kernel from the committed PMC summary of
    this config (tools/pmc_flops.py over one rocprofv3 --pmc pass of this same
    command; profiles/), or {}."""
    path = _profile_path(f"pmc_flops_{config}.json")
    try:
        with open(path) as f:
            return json.load(f)["kernels"]
    except (OSError, ValueError, KeyError):
        return {}


def _flops_of(table, prefixes):
    tot = [v["fp64_flops"] for k, v in table.items() if any(k.startswith(p) for p in prefixes)]
    return sum(tot) if tot else None


def cg_bytes(num_obs, num_points, num_frames, ng, dist_sizes):
    """Algorithmic bytes of one CG iteration (one implicit-Schur product + the
    vector updates) of a reprojection-only problem, DESIGN.md §5 "BA roofline":
      per observation  136 B  pass A: slot record (landmark + Cauchy weight) 32,
                              point-order slot 4, c_o store 32; k_point_w: c_o 32;
                              pass B: point index 4, slot record 32
      per point        152 B  k_point_w: CSR start 8, V 48, D 24, free flag 8,
                              w store 32; pass B: w read once 32
      per frame               pass B: world_to_cam + 22 generators (144 doubles);
                              update frame blocks: the 22 generators (132 doubles);
                              pass A: projection record (18 + K doubles); direction
                              records dz, dp (read) and the combined one (written,
                              read by pass B): 4 x (9 + live distortion) doubles
      per camera entry 704 B  replica sum: 32 replicas read + re-zeroed (512),
                              damping, z, p_old, p_new, y (48); update: entry
                              descriptor 16, x r/w 16, p, q, b, r_in, r_out, z (48),
                              block-inverse row (8 per block entry, ~7)
    Gathers that re-read L2-resident tables (the w of a point per observation,
    the frame records per wave) are counted once."""
    k = max(int(x) for x in dist_sizes) if len(dist_sizes) else 0
    live = k // 2 if k > 5 else k
    per_frame = 8 * (144 + 132 + (18 + k) + 4 * (9 + live))
    return 136 * num_obs + 152 * num_points + per_frame * num_frames + 704 * ng


def _ba_summary(config):
    """Committed CG-iteration summary of this config (tools/ba_roofline.py over a
    rocprofv3 kernel trace + FETCH/WRITE/SQ passes of this same command), or {}."""
    path = _profile_path(f"ba_{config}.json")
    try:
        with open(path) as f:
            d = json.load(f)
        d["path"] = os.path.relpath(path, os.path.dirname(os.path.abspath(__file__)))
        return d
    except (OSError, ValueError):
        return {}


def ceres_surface(ev, P, torch, args):
    """What BracketedCamBatch::Refresh does per PrepareForEvaluation: upload the
    host parameter arrays (mvba_set_params), evaluate, rewrite the planes as
    insertion-order rows on the device (k_rows, Cauchy corrector applied) and
    copy them to pinned host memory (mvba_evaluate_packed, default transfer set
    = every non-constant block). Timed end to end on the host clock; the PCIe
    ceiling is a plain device-to-pinned copy of the same bytes."""
    from multiview_amd.evaluator import PinnedBuffer

    n = ev.num_residuals
    off = ev.set_transfer_blocks(None)
    packed = int(off[-1])
    reps = max(3, min(args.steps, 10))
    out = {}
    with PinnedBuffer(packed) as buf, PinnedBuffer(2 * n) as rbuf:
        def run(jac):
            # as the adapter: residuals and rows into pinned memory, no cost
            # (Ceres sums the cost from the residuals itself)
            ev.set_params()
            ev.evaluate_packed(jacobian=jac, apply_loss=True, out=buf.array if jac else None,
                               res_out=rbuf.array, want_cost=False)

        for jac in (True, False):
            run(jac)
            t0 = time.perf_counter()
            for _ in range(reps):
                run(jac)
            dt = (time.perf_counter() - t0) / reps
            nbytes = 8.0 * (packed * jac + 2 * n)  # rows + residuals
            out["jacobian" if jac else "residuals_only"] = {
                "evals_per_s": n / dt, "ms": 1e3 * dt, "bytes_to_host": nbytes,
                "achieved_GBps": nbytes / dt / 1e9}
    # achievable device -> pinned host rate for the same byte count
    nb = int(8 * packed)
    d = torch.empty(nb, dtype=torch.uint8, device="cuda")
    h = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    h.copy_(d)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        h.copy_(d)
    torch.cuda.synchronize()
    copy_gbs = nb / ((time.perf_counter() - t0) / reps) / 1e9
    del d, h
    # the same evaluation into pageable numpy memory (staged through pinned buffers)
    ev.evaluate(jacobian=True, apply_loss=True)
    t0 = time.perf_counter()
    for _ in range(reps):
        ev.set_params()
        ev.evaluate(jacobian=True, apply_loss=True)
    full_dt = (time.perf_counter() - t0) / reps
    j = out["jacobian"]
    return {
        "what": "Ceres-surface hand-over per evaluation point: mvba_set_params (host arrays) + "
                "evaluate + device transposition into AddResidualBlock-order rows (Cauchy "
                "corrector) + one device-to-pinned copy (mvba_evaluate_packed)",
        "evals_per_s": j["evals_per_s"],
        "ms": j["ms"],
        "packed_doubles": packed,
        "pcie_GBps": j["achieved_GBps"],
        "pcie_copy_GBps": copy_gbs,
        "frac_of_copy": j["achieved_GBps"] / copy_gbs,
        "pcie_spec_GBps": 64.0,
        "residuals_only": out["residuals_only"],
        "pageable_full_layout": {"evals_per_s": n / full_dt, "ms": 1e3 * full_dt,
                                 "note": "mvba_evaluate into pageable numpy arrays (Ceres jac_stride "
                                         "layout, zero-filled), staged through two pinned 32 MB buffers"},
    }


def mesh_bench(torch, stream, nrays, args):
    """--mesh path (meshTriangulations -> ray_mesh_intersect, texture_processing.cc:
    1436-1479, 1566-1625): closest hits of one ray per observation against an
    icosphere of the scene's size (subdivision level --mesh-subdiv), rays grouped
    by camera as meshTriangulations issues them (image-major order), timed on the
    launch stream; the host BVH build (loadMeshBuildTree's tree) timed beside."""
    from multiview_amd import rig
    from multiview_amd.tracks import Mesh

    V, F = rig.sphere_mesh(args.mesh_subdiv)
    t0 = time.perf_counter()
    M = Mesh(V, F)
    build_s = time.perf_counter() - t0
    info = M.info()
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    ncam = 3000
    per = (nrays + ncam - 1) // ncam
    phi = torch.rand(ncam, device="cuda", generator=g, dtype=torch.float64) * 2 * np.pi
    C = torch.stack([8 * torch.cos(phi), 0.3 * torch.sin(3 * phi), 8 * torch.sin(phi)], 1)
    v = torch.randn(ncam, per, 3, device="cuda", generator=g, dtype=torch.float64)
    v = v / v.norm(dim=2, keepdim=True)
    v = torch.where(((v * C[:, None, :]).sum(2, keepdim=True) < 0), -v, v)  # the side the camera sees
    d = rig.SPHERE_RADIUS * v - C[:, None, :]
    d = d / d.norm(dim=2, keepdim=True)
    o = C[:, None, :].expand(ncam, per, 3).reshape(-1, 3)[:nrays].float().contiguous()
    d = d.reshape(-1, 3)[:nrays].float().contiguous()
    t = torch.empty(nrays, dtype=torch.float32, device="cuda")
    f = torch.empty(nrays, dtype=torch.int32, device="cuda")
    sh = stream.cuda_stream
    for _ in range(args.warmup):
        M.intersect_device(o, d, 0.0, 100.0, t, f, stream=sh)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(args.steps):
        M.intersect_device(o, d, 0.0, 100.0, t, f, stream=sh)
    e1.record(stream)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    hit = float((f >= 0).float().mean().item())
    M.close()
    return {
        "what": "closest-hit ray-mesh intersection (BVH traversal, rayint's float triangle test), one ray per "
                "observation, 3000 cameras",
        "rays": nrays, "faces": int(F.shape[0]), "bvh_nodes": info["num_nodes"], "bvh_depth": info["depth"],
        "rays_per_s": nrays / (ms * 1e-3), "kernel_ms": ms, "hit_fraction": hit,
        "bvh_build_s": build_s,
        "bound": "latency (dependent node loads per ray; node + triangle sets of "
                 f"{(32 * info['num_nodes'] + 48 * int(F.shape[0])) / 1e6:.1f} MB stay in the on-die caches)",
    }


def main():
    args = parse()
    rc = maybe_launch(args)
    if rc is not None:
        raise SystemExit(rc)
    import torch
    import torch.distributed as dist

    from multiview_amd import _lib, rig
    from multiview_amd.evaluator import Evaluator

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        # the LM phase captures its CG runs with the ncclAllReduce inside
        # (mvba_solve.cpp cg_device): no user-buffer registration of captured
        # collectives (56 KB exchanges gain nothing from zero-copy, and the
        # registration would map the solver's buffers to every peer)
        os.environ.setdefault("NCCL_GRAPH_REGISTER", "0")
        local = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local)
        from datetime import timedelta

        tmo = timedelta(seconds=args.dist_timeout)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
        else:
            dist.init_process_group(args.dist_backend, timeout=tmo)
        # control group on the CPU: ranks agree on phase failures over it,
        # whatever state the RCCL communicators are in. A failing rank may wait
        # there while a peer is still inside a collective that only its own
        # timeout (--dist-timeout) or the LM watchdog (--ba-deadline) ends, so
        # its timeout covers both.
        ctrl = dist.new_group(backend="gloo", timeout=timedelta(
            seconds=2 * args.dist_timeout + args.ba_deadline + 60))
    else:
        torch.cuda.set_device(0)
        ctrl = None
    dev = torch.cuda.current_device()

    cfg = dict(rig.CONFIGS[args.config])
    npts = cfg["num_points"]
    flags = rig.FloatFlags(**rig.CONFIG_FLAGS.get(args.config, {}))
    strong = args.scaling == "strong"
    # the committed per-launch PMC summaries (K1 traffic, fp64 counts, the CG
    # iteration's kernels) were measured on the whole config on one GPU: they
    # apply to this line only when it runs exactly that workload
    whole_cfg = summaries_apply(world, args.shard_of)

    def shard_cfg(strong_split):
        c = dict(cfg)
        if strong_split:
            # the config's whole problem (make_strong_shard cuts it)
            c["point_range"] = (0, npts)
        else:
            # each rank owns a config-sized shard of an N x larger problem
            c["point_range"] = (rank * npts, (rank + 1) * npts)
        return c

    def make_strong_shard():
        # the config's landmarks split into contiguous ranges of capture order
        # (rig.shard_points): every rank generates the whole problem and keeps
        # its range, so the shards partition exactly the N = 1 workload
        split = world if world > 1 else max(1, args.shard_of)
        R = rig.make_rig(**shard_cfg(True))
        return R if split == 1 else rig.shard_points(R, rank, split)

    t0 = time.perf_counter()
    R = make_strong_shard() if strong else rig.make_rig(**shard_cfg(False))
    P = rig.build_problem(R, flags)
    t_gen = time.perf_counter() - t0

    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream

    def time_eval(ev):
        """W warm-up + K timed evaluation steps (barrier + synchronize on both
        sides, max over ranks). Returns (max seconds, all ranks' evals, prep ms,
        K1 ms, planes)."""
        n = ev.num_residuals
        ld = ev.ld
        res = torch.empty((2, ld), dtype=torch.float64, device="cuda")
        jac = torch.empty((ev.stride, ld), dtype=torch.float64, device="cuda")

        def step(events=None):
            if events is None:
                ev.evaluate_device(True, residuals=res, jac=jac, ld=ld, stream=sh)
            else:
                events[0].record(stream)
                ev.evaluate_device(True, residuals=res, jac=jac, ld=ld, stream=sh, phase=_lib.EVAL_PREP_ONLY)
                events[1].record(stream)
                ev.evaluate_device(True, residuals=res, jac=jac, ld=ld, stream=sh, phase=_lib.EVAL_SKIP_PREP)
                events[2].record(stream)

        for _ in range(args.warmup):
            step()
        ev.sync(sh)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        le = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        t0 = time.perf_counter()
        le[0].record(stream)
        for k in range(args.steps):
            step()
        le[1].record(stream)
        t_issue = time.perf_counter() - t0  # host time to enqueue the K steps
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        ev.sync(sh)  # raises on device-side errors (alpha out of range, fused wait given up)
        # Per-launch times, from the same K steps run again with HIP events on
        # the launch stream (events between kernels cost the step ~10 us, c2 114
        # vs 104 us, tools/step_overhead.py, so the timed loop above has none):
        # (1) the launch the timed loop runs (one k_eval / k_eval_local launch
        # for a one-model problem, mvba_eval_form), events around each step;
        # (2) the split form beside it: the prep launch, then K1 (k_obs) alone.
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.steps)]
        for k in range(args.steps):
            evs[k][0].record(stream)
            step()
            evs[k][1].record(stream)
        torch.cuda.synchronize()
        ev.sync(sh)
        launch_event_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
        # GPU time per step of the timed loop itself: two events bracketing its K
        # back-to-back steps (for a one-launch form: the launch's average duration
        # with the boundary to the next launch)
        launch_ms = le[0].elapsed_time(le[1]) / args.steps
        time_eval.launch_event_ms = launch_event_ms
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
        for k in range(args.steps):
            step(evs[k])
        torch.cuda.synchronize()
        ev.sync(sh)
        prep_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
        obs_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        tot = torch.tensor([float(n)], dtype=torch.float64, device="cuda")
        per_rank = None
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dist.all_reduce(tot, op=dist.ReduceOp.SUM)
            mine = torch.tensor([1e3 * dt / args.steps, prep_ms, obs_ms, float(n), 1e3 * t_issue / args.steps,
                                 launch_ms], dtype=torch.float64, device="cuda")
            allr = [torch.empty_like(mine) for _ in range(world)]
            dist.all_gather(allr, mine)
            rows = [r.cpu().tolist() for r in allr]
            per_rank = {"ms_per_step": [r[0] for r in rows], "launch_ms": [r[5] for r in rows],
                        "split_prep_ms": [r[1] for r in rows], "split_k1_ms": [r[2] for r in rows],
                        "num_residuals": [int(r[3]) for r in rows],
                        "host_issue_ms_per_step": [r[4] for r in rows]}
        del res, jac
        time_eval.host_issue_ms = 1e3 * t_issue / args.steps
        return float(t.item()), float(tot.item()) * args.steps, prep_ms, obs_ms, launch_ms, per_rank

    ev = Evaluator(P, device=dev)
    ev.set_params()
    n = ev.num_residuals
    dt_max, total_evals, prep_ms, obs_ms, launch_ms, per_rank = time_eval(ev)

    if world == 1 and args.shard_of > 1:  # timing rehearsal, not a bench line
        cfg["shard_rehearsal"] = f"rank 0's shard of a {args.shard_of}-way landmark split, one process"
    form = ev.eval_form()
    model = cfg["models"][0]
    bytes_eval = ev.eval_bytes(True)                 # algorithmic bytes of K1 per launch set
    bytes_prep = ev.eval_bytes_prep()                # the prep's (landmark gather + K0 frame records)
    k1_achieved = bytes_eval / (obs_ms * 1e-3) / 1e9
    if form == _lib.FORM_SPLIT:
        # several camera models: the timed step is the prep launch + one K1 launch
        # per model group; the roofline is K1's
        kname, kernel_ms, bytes_launch, traffic_kind = f"k_obs<{model}> (K1)", obs_ms, bytes_eval, "k1"
    else:
        kname = f"{_lib.FORM_NAMES[form]}<{model}>"
        kernel_ms, bytes_launch, traffic_kind = launch_ms, bytes_eval + bytes_prep, "eval"
    achieved = bytes_launch / (kernel_ms * 1e-3) / 1e9    # GB/s
    line = {
        "metric": "residual+Jacobian evals/sec (3-cam rig, 1M obs)",
        "value": total_evals / dt_max,
        "unit": "evals/s",
        "n_gpus": world,
        "devices": min(world, torch.cuda.device_count()),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * dt_max / args.steps,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (deterministic rig generator, multiview_amd/rig.py)",
        "config": {
            "workload": f"{args.config}: {cfg['num_sensors']}-sensor rig, "
                        + (f"{npts} landmarks split over {world} landmark-range shard(s), " if strong
                           else f"{npts} landmarks x {world} shard(s), ")
                        + f"{n} obs/GPU, "
                        f"{cfg['models'][0]} distortion, all blocks floating, fp64",
            "num_residuals_per_gpu": n,
            "num_frames": ev.num_frames,
            "num_points_per_gpu": ev.num_points,
            "parallelism": f"landmark-range shards x{world}",
            **({"shard_rehearsal": cfg["shard_rehearsal"]} if "shard_rehearsal" in cfg else {}),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": kname,
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": _pmc_traffic(args.config, traffic_kind) if whole_cfg else None,
            **({} if whole_cfg else {"traffic_note": "null: the committed PMC summaries (profiles/) are per "
                                     "launch of the whole single-GPU config, not of this rank's shard"}),
            "bytes_per_launch": bytes_launch,
            "bytes_note": "K1's algorithmic bytes (per observation 16 meas + 4 point index + 24 landmark + 16 "
                          "residual + 16 per written Jacobian column)"
                          + ("" if form == _lib.FORM_SPLIT else
                             " + the prep's in the same launch (per landmark 65, per frame 1,456)"),
            "kernel_ms": kernel_ms,
            "kernel_timing": ("two HIP events on the launch stream bracketing the timed loop's K back-to-back "
                              "launches (the launch the loop runs, mvba_eval_form; per launch, boundary included)"
                              if form != _lib.FORM_SPLIT else
                              "HIP events on the launch stream around the K1 launch of K instrumented steps run "
                              "right after the timed loop"),
            "kernel_ms_event_per_launch": time_eval.launch_event_ms,
            "event_per_launch_note": "the same launch timed with events around each of K instrumented steps after "
                                     "the timed loop (each event pair adds ~2-4 us)",
            "split_form": {
                "what": "the same evaluation as two launches (prep, then K1 = k_obs), event-timed",
                "kernel": f"k_obs<{model}> (K1)",
                "kernel_ms": obs_ms,
                "prep_ms": prep_ms,
                "bytes_per_launch": bytes_eval,
                "achieved": k1_achieved,
                "frac": k1_achieved / HBM_PEAK_GBS,
                "traffic": _pmc_traffic(args.config, "k1") if whole_cfg else None,
            },
        },
        "gen_s": t_gen,
        # host time to enqueue one step (Python + ctypes + the launches): when it
        # approaches ms_per_step the step is launch-bound, not GPU-bound
        "host_issue_ms_per_step": time_eval.host_issue_ms,
    }
    if per_rank is not None:
        line["per_rank"] = per_rank
    # achievable HBM bandwidth on this box ("measure achieved peak
    # with a STREAM-like copy kernel ... and report against both")
    stream_gbs = _stream_copy_gbs(torch, stream)
    line["roofline"]["stream_copy_gbs"] = stream_gbs
    line["roofline"]["frac_of_stream"] = achieved / stream_gbs if stream_gbs else None
    line["roofline"]["stream_note"] = "1 GiB device-to-device tensor copy (read + write bytes), same stream"
    # fp64 arithmetic of the same launch (PMC instruction counts): the second
    # roofline, to name the binding resource
    flops_tab = _pmc_flops(args.config) if whole_cfg else {}
    if form == _lib.FORM_SPLIT:
        k1_flops = next((v["fp64_flops"] for k, v in flops_tab.items()
                         if k.startswith("mvba::k_obs<") and k.endswith("double>")), None)
    else:
        pre = "mvba::k_eval<" if form == _lib.FORM_FUSED else "mvba::k_eval_local<"
        k1_flops = next((v["fp64_flops"] for k, v in flops_tab.items()
                         if k.startswith(pre) and k.endswith("double, true>")), None)
    if k1_flops is not None:
        tf = k1_flops / (kernel_ms * 1e-3) / 1e12
        line["roofline"]["fp64_flops_per_launch"] = k1_flops
        line["roofline"]["fp64_tflops"] = tf
        line["roofline"]["fp64_peak_tflops"] = FP64_PEAK_TFLOPS
        line["roofline"]["fp64_frac"] = tf / FP64_PEAK_TFLOPS
        line["roofline"]["binding"] = "hbm" if achieved / HBM_PEAK_GBS >= tf / FP64_PEAK_TFLOPS else "fp64"
    # ---- depth blocks (c5): K1-depth evaluation, materialised
    if ev.num_depth > 0:
        dld = (ev.num_depth_slots + 63) // 64 * 64
        dres = torch.empty((3, dld), dtype=torch.float64, device="cuda")
        dJ = torch.empty((_lib.DJAC_ROWS, dld), dtype=torch.float64, device="cuda")

        def dstep():
            _lib.check(ev.lib.mvba_evaluate_depth_device(
                ev.h, _lib.EVAL_RESIDUALS | _lib.EVAL_JACOBIAN | _lib.EVAL_SKIP_PREP, 0.0,
                C.c_void_p(dres.data_ptr()), C.c_void_p(dJ.data_ptr()), dld, C.c_void_p(sh)), ev.h)

        for _ in range(args.warmup):
            dstep()
        torch.cuda.synchronize()
        de = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        de[0].record(stream)
        for _ in range(args.steps):
            dstep()
        de[1].record(stream)
        torch.cuda.synchronize()
        d_ms = de[0].elapsed_time(de[1]) / args.steps
        dbytes = float(ev.lib.mvba_eval_bytes(ev.h, _lib.EVAL_DEPTH))
        line["depth"] = {
            "what": "BracketedDepthError residual+Jacobian (K1-depth, materialised, column planes)",
            "kernel": "k_depth_obs<double>",
            "num_depth_residuals": ev.num_depth,
            "evals_per_s": ev.num_depth / (d_ms * 1e-3),
            "kernel_ms": d_ms,
            "bytes_per_launch": dbytes,
            "achieved_GBps": dbytes / (d_ms * 1e-3) / 1e9,
            "frac_of_hbm_peak": dbytes / (d_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            # HBM bytes per launch from the committed FETCH / WRITE passes of this
            # config (pmc_depth_<cfg>.json) and its fp64 work (pmc_flops_<cfg>.json)
            "traffic": _pmc_traffic(args.config, "depth") if whole_cfg else None,
        }
        d_flops = next((v["fp64_flops"] for k, v in flops_tab.items() if k.startswith("mvba::k_depth_obs<double>")),
                       None)
        if d_flops is not None:
            dtf = d_flops / (d_ms * 1e-3) / 1e12
            line["depth"].update({"fp64_flops_per_launch": d_flops, "fp64_tflops": dtf,
                                  "fp64_frac": dtf / FP64_PEAK_TFLOPS,
                                  "binding": "hbm" if dbytes / (d_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
                                  >= dtf / FP64_PEAK_TFLOPS else "fp64"})

    # ---- fp32 evaluation (config c5 is quoted "fp32 eval / fp64 solve"): the same
    # fp64 arithmetic, outputs rounded to float at the store (half the output bytes)
    ld = ev.ld
    res32 = torch.empty((2, ld), dtype=torch.float32, device="cuda")
    jac32 = torch.empty((ev.stride, ld), dtype=torch.float32, device="cuda")
    for _ in range(args.warmup):
        ev.evaluate_device(True, residuals=res32, jac=jac32, ld=ld, stream=sh, phase=_lib.EVAL_SKIP_PREP)
    torch.cuda.synchronize()
    fe = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fe[0].record(stream)
    for _ in range(args.steps):
        ev.evaluate_device(True, residuals=res32, jac=jac32, ld=ld, stream=sh, phase=_lib.EVAL_SKIP_PREP)
    fe[1].record(stream)
    torch.cuda.synchronize()
    f_ms = fe[0].elapsed_time(fe[1]) / args.steps
    reads = 44.0 * n  # meas 16 + point index 4 + landmark 24 per observation
    f32_bytes = reads + (bytes_eval - reads) / 2.0
    line["eval_f32"] = {
        "what": "K1 with fp32 outputs (fp64 arithmetic, one rounding at the store)",
        "evals_per_s": n / (f_ms * 1e-3),
        "kernel_ms": f_ms,
        "bytes_per_launch": f32_bytes,
        "achieved_GBps": f32_bytes / (f_ms * 1e-3) / 1e9,
    }
    del res32, jac32
    if ev.num_depth > 0:
        dres32 = torch.empty((3, dld), dtype=torch.float32, device="cuda")
        dJ32 = torch.empty((_lib.DJAC_ROWS, dld), dtype=torch.float32, device="cuda")

        def dstep32():
            _lib.check(ev.lib.mvba_evaluate_depth_device_f32(
                ev.h, _lib.EVAL_RESIDUALS | _lib.EVAL_JACOBIAN | _lib.EVAL_SKIP_PREP, 0.0,
                C.c_void_p(dres32.data_ptr()), C.c_void_p(dJ32.data_ptr()), dld, C.c_void_p(sh)), ev.h)

        for _ in range(args.warmup):
            dstep32()
        torch.cuda.synchronize()
        fe[0].record(stream)
        for _ in range(args.steps):
            dstep32()
        fe[1].record(stream)
        torch.cuda.synchronize()
        fd_ms = fe[0].elapsed_time(fe[1]) / args.steps
        dreads = 56.0 * ev.num_depth
        line["eval_f32"]["depth_evals_per_s"] = ev.num_depth / (fd_ms * 1e-3)
        line["eval_f32"]["depth_kernel_ms"] = fd_ms
        line["eval_f32"]["depth_achieved_GBps"] = (dreads + (dbytes - dreads) / 2.0) / (fd_ms * 1e-3) / 1e9
        del dres32, dJ32

    # ---- the Ceres-surface hand-over (include/mvba/ceres_surface.h): host
    # parameters in, AddResidualBlock-order rows out through one PCIe copy
    if world == 1:
        line["ceres_surface"] = ceres_surface(ev, P, torch, args)

    # ---- phase B: normal equations (K2) + the per-iteration exchange (§8e)
    from multiview_amd.dist import NormalEquationBuffer, check_layouts_agree

    L = ev.lin_layout()

    def phase_lin():
        lin = None
        if L["supported"]:
            if world > 1:
                check_layouts_agree(L, P.block_size, device="cuda")
            buf = NormalEquationBuffer(L, device="cuda")
            pg = torch.empty(3 * L["num_points"], dtype=torch.float64, device="cuda")
            ph = torch.empty(6 * L["num_points"], dtype=torch.float64, device="cuda")

            def lin_step(events=None):
                if events is not None:
                    events[0].record(stream)
                ev.linearize_device(buf.grad, buf.hess, pg, ph, buf.cost, apply_loss=True,
                                    robust_threshold=3.0, stream=sh)
                if events is not None:
                    events[1].record(stream)
                if world > 1:
                    buf.allreduce()
                if events is not None:
                    events[2].record(stream)

            for _ in range(args.warmup):
                lin_step()
            torch.cuda.synchronize()
            levs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(args.steps):
                lin_step(levs[k])
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            ldt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
            if world > 1:
                dist.all_reduce(ldt, op=dist.ReduceOp.MAX)
            ev.sync(sh)
            lin_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in levs]))
            ar_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in levs]))
            lin = {
                "what": "K2 linearization (Cauchy-corrected J^T r, block-diagonal J^T J: camera side "
                        "via fp64 MFMA Gram + in-block expansion, point side on a second stream) + RCCL "
                        "all-reduce of the camera blocks",
                "evals_per_s": total_evals / float(ldt.item()),
                "ms_per_step": 1e3 * float(ldt.item()) / args.steps,
                "kernel_ms": lin_ms,
                "allreduce_ms": ar_ms if world > 1 else 0.0,
                "allreduce_bytes": buf.payload_bytes if world > 1 else 0,
                "cam_params": L["cam_grad_size"],
            }

            # the two sides timed alone (same stream, HIP events, parameters and K0
            # records unchanged): camera side = k_frame_lin + replica reduce,
            # point side = k_points_lin on the library's second stream
            def side_ms(side):
                kw = dict(apply_loss=True, robust_threshold=3.0, stream=sh, skip_prep=True, side=side)
                for _ in range(args.warmup):
                    ev.linearize_device(buf.grad, buf.hess, pg, ph, buf.cost, **kw)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(args.steps):
                    ev.linearize_device(buf.grad, buf.hess, pg, ph, buf.cost, **kw)
                e1.record(stream)
                e1.synchronize()
                return e0.elapsed_time(e1) / args.steps

            cam_ms, pts_ms = side_ms("camera"), side_ms("points")
            # what an LM iteration pays: after a successful step the solver
            # linearizes at the candidate whose frame records its evaluation
            # already stored (SKIP_PREP: both sides, no prep launch)
            lin["kernel_ms_records_current"] = side_ms("both")
            lin["records_current_note"] = ("K2 + replica reduce with the frame records current (SKIP_PREP), as "
                                           "mvba_solve linearizes after a successful LM step; kernel_ms includes "
                                           "the prep launch (first linearization at a new point)")
            mfma = float(ev.lib.mvba_lin_mfma_flops(ev.h))
            lin["camera_side_ms"] = cam_ms
            lin["point_side_ms"] = pts_ms
            # X1 evidence (north_star: MFMA for the dense normal-equation blocks):
            # fp64 MFMA work issued by the camera-side Gram kernel against the
            # MI355X fp64 matrix peak, over the camera side's time
            lin["mfma"] = {
                "kernel": "k_frame_lin (v_mfma_f64_16x16x4f64)",
                "flops_per_launch": mfma,
                "achieved_tflops": mfma / (cam_ms * 1e-3) / 1e12,
                "peak_tflops": FP64_PEAK_TFLOPS,
                "util": mfma / (cam_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                "note": "issued MFMA flops (zero-padded tile columns included) / camera-side time "
                        "(Gram + expansion + replica reduce)",
            }
            # fused mode: 48 B per evaluation (observation record +
            # landmark) against the fp64 work of the linearization kernels
            # the fused launch is k_frame_lin<model, deg, POINTS = true> (point side as
            # extra blocks of the same launch); the POINTS = false variant and
            # k_points_lin belong to the camera-only / point-only phases timed above
            fused = {k: v for k, v in flops_tab.items()
                     if k.startswith(("mvba::k_prep", "mvba::k_rep_reduce"))
                     or (k.startswith("mvba::k_frame_lin<") and k.endswith("true>"))}
            lin_flops = _flops_of(fused, [""]) if fused else None
            lin_bytes = 48.0 * n
            lin["hbm_bytes"] = lin_bytes
            lin["hbm_frac"] = lin_bytes / (lin_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
            if lin_flops is not None:
                tf = lin_flops / (lin_ms * 1e-3) / 1e12
                lin["fp64_flops"] = lin_flops
                lin["fp64_mfma_flops"] = sum(v["fp64_mfma_flops"] for v in fused.values())
                lin["fp64_tflops"] = tf
                lin["fp64_frac"] = tf / FP64_PEAK_TFLOPS
                lin["bound_us"] = 1e6 * max(lin_bytes / (HBM_PEAK_GBS * 1e9), lin_flops / (FP64_PEAK_TFLOPS * 1e12))
                lin["binding"] = "fp64" if lin_flops / FP64_PEAK_TFLOPS / 1e12 > lin_bytes / HBM_PEAK_GBS / 1e9 else "hbm"
        line["linearize"] = lin


    # ---- phase C: Levenberg-Marquardt (mvba_solve: ITERATIVE_SCHUR replacement)
    def phase_ba():
        if L["supported"] and args.ba_iters > 0:
            from multiview_amd.dist import Comm, SolverExchange

            comm = ex = None
            if world > 1:
                if args.dist_backend == "nccl":
                    # library-native RCCL, stream-ordered exchange; non-blocking
                    # communicator whose init and enqueues fail past the deadline
                    comm = Comm.rccl(dev, timeout_s=args.ba_deadline)
                else:
                    ex = SolverExchange(device=dev)  # gloo rehearsal: host-staged exchange
            elif args.ba_exchange == "rccl":
                # one-rank RCCL communicator: the sharded solve's code path
                # (exchange enqueues, fold-mode CG tail, captured CG runs with
                # the all-reduce inside), timed on one GPU
                comm = Comm.rccl_world1(dev, timeout_s=args.ba_deadline)
            inject = injected_failure(os.environ.get("MVBA_BENCH_INJECT", ""), rank)
            if inject and ex is not None:
                ex = FailingExchange(ex)
            elif inject and comm is not None:
                comm.abort()  # this rank's exchanges fail; its peers meet the deadline
            with comm_lock:
                resources["comm"] = comm
            solve_kw = dict(max_num_iterations=args.ba_iters, function_tolerance=0.0, gradient_tolerance=0.0,
                            parameter_tolerance=0.0, use_loss=1, robust_threshold=3.0, allreduce=ex, comm=comm)
            # warm-up: one untimed solve of the same length from the same start
            # (allocation, and the CG runs / step graphs captured once per handle,
            # as a long rig_calibrator solve captures them in its first LM steps)
            ev.set_params()
            ev.solve(**solve_kw, stream=sh)
            ev.set_params()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            s = ev.solve(**solve_kw, stream=sh)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            bdt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
            if world > 1:
                dist.all_reduce(bdt, op=dist.ReduceOp.MAX)
            iters = max(s["num_iterations"], 1)
            line["ba"] = {
                "what": "LM iterations (Ceres-1.14 trust region, Jacobi scaling, implicit-Schur PCG with "
                        "block-Jacobi preconditioner, Cauchy loss 3.0), all blocks floating",
                "iters_per_s": iters / float(bdt.item()),
                "warmup": "one untimed solve of the same length from the same start (allocation, graph captures)",
                "ms_per_iter": 1e3 * float(bdt.item()) / iters,
                "lm_iterations": s["num_iterations"],
                "successful_steps": s["num_successful_steps"],
                "cg_iterations": s["num_linear_iterations"],
                # pass B / K2 accumulate shared camera entries with fp64 atomics, so
                # the CG count (and LM it/s) varies run to run; this one does not
                "ms_per_cg_iteration": 1e3 * s["linear_solver_time_s"] / max(s["num_linear_iterations"], 1),
                "linearize_s": s["linearize_time_s"],
                "linear_solver_s": s["linear_solver_time_s"],
                "eval_s": s["eval_time_s"],
                "initial_cost": s["initial_cost"],
                "final_cost": s["final_cost"],
                "exchange": ("rccl (mvba_comm_allreduce, stream-ordered)" if comm and world > 1 else
                             "rccl (one-rank communicator: the sharded path rehearsed, mvba_comm_allreduce)"
                             if comm else "gloo (host-staged callback)" if ex else "none (single rank)"),
                "exchange_calls": ex.calls if ex else None,
                # captured CG runs replayed (0: every CG kernel and exchange launched eagerly)
                "cg_graph_launches": s.get("cg_graph_launches"),
            }
            if ev.num_depth == 0:
                cgb = cg_bytes(ev.num_residuals, int(L["num_points"]), ev.num_frames, int(L["cam_grad_size"]),
                               P.camera_dist_size)
                wall_ms = line["ba"]["ms_per_cg_iteration"]
                roof = {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
                        "bytes_per_cg_iteration": cgb,
                        "achieved_wall": cgb / (wall_ms * 1e-3) / 1e9,
                        "frac_wall": cgb / (wall_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                        "wall_note": "algorithmic bytes / (linear-solver wall time / CG iterations): includes the "
                                     "residual-reset products (every 10th), the per-solve setup and host reads"}
                # the whole config's summary, or the one-GPU shard rehearsal's own
                # (ba_<cfg>_s<N>[_rccl].json: the rank-0 shard through the same exchange)
                ba_key = (args.config if whole_cfg else
                          f"{args.config}_s{args.shard_of}{'_rccl' if comm is not None else ''}"
                          if world == 1 and args.shard_of > 1 else None)
                summ = _ba_summary(ba_key) if ba_key else {}
                if summ:
                    kus = summ["kernel_us_per_cg_iteration"]
                    roof.update({
                        "kernel_us": kus,
                        "achieved": cgb / (kus * 1e-6) / 1e9,
                        "frac": cgb / (kus * 1e-6) / 1e9 / HBM_PEAK_GBS,
                        "traffic": summ["traffic_bytes_per_cg_iteration"],
                        "traffic_ratio": summ["traffic_bytes_per_cg_iteration"] / cgb,
                        "valu_floor_us": summ["valu_floor_us"],
                        "valu_frac": summ["valu_floor_us"] / kus,
                        "source": summ["path"] + " (rocprofv3 kernel trace: median span of non-gated iterations "
                                  "pass A -> update, or the fused step's period, boundaries included; FETCH_SIZE x2 "
                                  "+ WRITE_SIZE and SQ_INSTS_VALU per kernel, median of non-gated launches)",
                        "cg_form": summ.get("cg_form", "separate update"),
                    })
                line["ba"]["roofline"] = roof
            if world > 1 or comm is not None:
                # the per-CG-iteration exchange alone: one all-reduce of the
                # camera-side product vector (cam_grad_size doubles), on the solver's
                # stream, HIP events around K of them
                ng = int(L["cam_grad_size"])
                vbuf = torch.ones(ng, dtype=torch.float64, device="cuda")

                def xchg():
                    if comm is not None:
                        comm.allreduce(vbuf.data_ptr(), ng, 0, sh)
                    else:
                        ex(vbuf.data_ptr(), ng, 0, sh)

                for _ in range(args.warmup):
                    xchg()
                torch.cuda.synchronize()
                if world > 1:
                    dist.barrier()
                xe = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                t0 = time.perf_counter()
                xe[0].record(stream)
                for _ in range(args.steps):
                    xchg()
                xe[1].record(stream)
                xe[1].synchronize()
                host_us = 1e6 * (time.perf_counter() - t0) / args.steps
                line["ba"]["exchange_us_per_cg_iteration"] = 1e3 * xe[0].elapsed_time(xe[1]) / args.steps
                line["ba"]["exchange_host_us_per_call"] = host_us
                line["ba"]["exchange_bytes_per_cg_iteration"] = 8 * ng
                del vbuf
            if world == 1:
                # deterministic mode (fixed-order slab gathers instead of fp64 atomics):
                # same LM iterations, reproducible CG count; its cost per CG iteration
                ev.set_params()
                ev.solve(**dict(solve_kw, deterministic=1), stream=sh)  # warm-up, as above
                ev.set_params()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                sd = ev.solve(**dict(solve_kw, deterministic=1), stream=sh)
                torch.cuda.synchronize()
                ddt = time.perf_counter() - t0
                line["ba_deterministic"] = {
                    "what": "the same LM run with mvba_solver_options.deterministic = 1",
                    "iters_per_s": max(sd["num_iterations"], 1) / ddt,
                    "cg_iterations": sd["num_linear_iterations"],
                    "ms_per_cg_iteration": 1e3 * sd["linear_solver_time_s"] / max(sd["num_linear_iterations"], 1),
                    "linearize_s": sd["linearize_time_s"],
                    "final_cost": sd["final_cost"],
                }
            take_comm_and_close()

    # ---- N > 1: the weak-scaling line as well (config-sized shard per rank)
    def phase_weak():
        nonlocal ev
        if world > 1 and strong:
            ev.close()
            Rw = rig.make_rig(**shard_cfg(False))
            Pw = rig.build_problem(Rw, flags)
            ev = Evaluator(Pw, device=dev)
            ev.set_params()
            wdt, wtot, _, _, w_launch_ms, w_per_rank = time_eval(ev)
            line["weak"] = {
                "what": f"weak scaling: every rank owns a {args.config}-sized shard of a {world} x larger problem",
                "value": wtot / wdt,
                "ms_per_step": 1e3 * wdt / args.steps,
                "num_residuals_per_gpu": ev.num_residuals,
                "kernel_ms": w_launch_ms,
                "per_rank": w_per_rank,
            }

    # Phases B and C (and the weak-scaling line) run guarded: an exception on
    # any rank, or an exchange that passes its deadline (the RCCL communicator is
    # non-blocking with a deadline, and a watchdog aborts it if the solve
    # overruns --ba-deadline), is recorded in the line under the phase's key and
    # the line still prints with the evaluation headline; every rank then skips
    # the phases that would need the others, and the process exits non-zero.
    # Ranks agree on failures over a gloo control group (CPU, independent of
    # RCCL state).
    guard = PhaseGuard(line, world, rank, ctrl)

    resources = {"comm": None}
    # the LM phase's watchdog (fire below) and the phase's own teardown both
    # reach the communicator: one lock, and the teardown takes the communicator
    # out of `resources` before closing it, so an abort never runs during or
    # after the close (Timer.cancel() does not wait for a fire() in progress)
    import threading

    comm_lock = threading.Lock()

    def take_comm_and_close():
        with comm_lock:
            c = resources.get("comm")
            resources["comm"] = None
        if c is not None:
            c.close()

    def phase_ba_watched():
        # watchdog: a solve that overruns the deadline (a peer that never joins
        # an exchange) has its communicator aborted from this thread, so the
        # pending collective returns and the solve raises instead of hanging
        def fire():
            with comm_lock:
                c = resources.get("comm")
                if c is not None:
                    print(f"bench.py: rank {rank}: LM phase past --ba-deadline {args.ba_deadline} s, aborting the "
                          "RCCL communicator", file=sys.stderr, flush=True)
                    c.abort()

        wd = threading.Timer(args.ba_deadline, fire) if world > 1 else None
        if wd is not None:
            wd.daemon = True
            wd.start()
        try:
            phase_ba()
        finally:
            if wd is not None:
                wd.cancel()
            take_comm_and_close()

    guard.run("linearize", phase_lin)
    if L["supported"] and args.ba_iters > 0:
        guard.run("ba", phase_ba_watched)
    if world > 1 and strong:
        guard.run("weak", phase_weak)

    if rank == 0 and world == 1 and args.mesh_subdiv > 0:
        line["mesh"] = mesh_bench(torch, stream, ev.num_residuals, args)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        print("[bench] cpu baseline", file=sys.stderr, flush=True)
        line["cpu_baseline"] = cpu_baseline(P, args.cpu_sample)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        # no rank exits (and has the launcher tear the others down) before rank 0
        # has printed
        dist.barrier(group=ctrl)
    ev.close()
    if world > 1:
        dist.destroy_process_group()
    if guard.errors:
        raise SystemExit(1)


if __name__ == "__main__":
    main()
