import os, sys
sys.path.insert(0, os.getcwd())
import torch, torch.multiprocessing as mp

def child(rank):
    from multiview_amd import _lib
    import ctypes as C
    lib = _lib.load(); n = C.c_int32(); lib.mvba_device_count(C.byref(n)); print("child", rank, n.value, flush=True)

if __name__ == "__main__":
    mode = sys.argv[1]
    if mode == "pre":
        torch.cuda.init(); print("parent pre-init count", torch.cuda.device_count(), flush=True)
    print("env HIP/ROCR/CUDA:", {k: v for k, v in os.environ.items() if "VISIBLE" in k}, flush=True)
    mp.spawn(child, nprocs=2, join=True)
    print("env after:", {k: v for k, v in os.environ.items() if "VISIBLE" in k}, flush=True)
    print("parent count", torch.cuda.device_count(), flush=True)
    x = torch.zeros(3, device="cuda"); print("ok", x.sum().item(), flush=True)
