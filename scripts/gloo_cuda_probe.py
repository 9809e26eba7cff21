"""Probe (GPU box): do gloo's reduce_scatter_tensor / all_gather_into_tensor take HIP tensors?
Two ranks on one GPU.  usage: python scripts/gloo_cuda_probe.py"""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def w(rank, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    x = torch.arange(8, dtype=torch.float32, device="cuda") * (rank + 1)
    out = torch.empty(4, device="cuda")
    res = {}
    try:
        dist.reduce_scatter_tensor(out, x)
        res["rs"] = out.tolist()
    except Exception as e:  # noqa: BLE001
        res["rs"] = f"ERR {type(e).__name__}: {e}"[:200]
    try:
        y = torch.empty(8, device="cuda")
        dist.all_gather_into_tensor(y, out)
        res["ag"] = y.tolist()
    except Exception as e:  # noqa: BLE001
        res["ag"] = f"ERR {type(e).__name__}: {e}"[:200]
    print(rank, res, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(w, args=(port,), nprocs=2)
    sys.exit(0)
