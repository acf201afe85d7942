"""Build libmvba.so (gfx950) in-tree with hipcc.

    python -m multiview_amd.build
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libmvba.so")
SOURCES = ["mvba_kernels.hip", "mvba_solver.hip", "mvba_depth.hip", "mvba_stats.hip", "mvba_tracks.hip",
           "mvba_mesh.hip", "mvba_rpc.hip", "mvba_comm.hip", "mvba_transfer.hip", "mvba_host.cpp", "mvba_transfer_host.cpp", "mvba_solve.cpp"]
# RCCL for the sharded solve's stream-ordered all-reduce (mvba_comm.hip). In a
# torch process the already loaded librccl.so.1 (same SONAME) is the one used.
LIBS = ["-L/opt/rocm/lib", "-lrccl"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-fopenmp", "-Wall",
         "-Wno-unused-function"]


def build(verbose: bool = False) -> str:
    from concurrent.futures import ThreadPoolExecutor

    headers = [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")] + \
        [os.path.join(HERE, "..", "include", "mvba", "mvba.h")]
    objs, cmds = [], []
    for src in SOURCES:
        obj = os.path.join(CSRC, os.path.splitext(src)[0] + ".o")
        srcp = os.path.join(CSRC, src)
        deps = [srcp] + headers
        if not os.path.exists(obj) or any(os.path.getmtime(d) > os.path.getmtime(obj) for d in deps):
            cmds.append([HIPCC] + FLAGS + ["-x", "hip", "-c", srcp, "-o", obj])
        objs.append(obj)
    jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", "8"))))

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)

    with ThreadPoolExecutor(jobs) as pool:
        list(pool.map(run, cmds))
    if not os.path.exists(OUT) or any(os.path.getmtime(o) > os.path.getmtime(OUT) for o in objs):
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fopenmp", "-o", OUT] + objs + LIBS
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
