"""Probe: can the library's RCCL communicator run world 2 on a one-GPU box?

Launched as `python -m torch.distributed.run --nproc-per-node 2 tools/rccl_probe.py`.
Both ranks bootstrap over gloo, join one mvba_comm RCCL communicator on
cuda:0, sum a device vector and check the result (rank r contributes r + 1 per
element). RCCL may refuse two ranks on one device ("duplicate GPU"); the probe
reports either outcome and exits 0 for a clean refusal, 1 for a wrong sum.
"""

import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from multiview_amd.dist import Comm  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    try:
        comm = Comm.rccl(0)
    except Exception as e:  # noqa: BLE001
        print(f"rank {rank}: RCCL communicator refused: {e}", flush=True)
        dist.barrier()
        dist.destroy_process_group()
        return 0
    n = 7041
    x = torch.full((n,), float(rank + 1), dtype=torch.float64, device="cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    comm.allreduce(x.data_ptr(), n, 0, s)
    torch.cuda.synchronize()
    want = world * (world + 1) / 2
    ok = bool(torch.all(x == want).item())
    print(f"rank {rank}: RCCL world {world} all-reduce sum {'ok' if ok else 'WRONG'} "
          f"(x[0] = {x[0].item()}, want {want})", flush=True)
    comm.close()
    dist.barrier()
    dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
