"""Diagnose the owned-RCCL communicator's init on one GPU (world 1), with RCCL's own log."""
import os
import socket
import sys

import torch
import torch.distributed as dist

from tensorflow_distributed_learning_amd import ops

C = ops.hip()
print("rccl version", C.RcclComm.version(), flush=True)
uid = C.RcclComm.unique_id()
print("uid bytes", len(uid), flush=True)
torch.cuda.set_device(0)
mode = sys.argv[1] if len(sys.argv) > 1 else "direct"
if mode == "pg":
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
c = C.RcclComm(uid, 0, 1, 0)
print("init ok", flush=True)
t = torch.ones(4, device="cuda")
c.all_reduce(t, 0)
torch.cuda.synchronize()
print("all_reduce ok", t.tolist(), flush=True)
c.abort()
print("abort ok", flush=True)
