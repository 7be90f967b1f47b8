"""Step-by-step bring-up of the native RCCL communicator (csrc/comm_bindings.cpp) with a print after every
call: the first tool when INA_COMM=native fails on a new box (run with NCCL_DEBUG=INFO)."""
import faulthandler
import os
import socket
import sys

faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from induction_network_on_fewrel_amd.ops._ext import ops  # noqa: E402


def p(*a):
    print(*a, flush=True)


o = ops()
p("ops loaded")
torch.cuda.init()
x = torch.zeros(4, device="cuda")
p("cuda ok", torch.cuda.get_device_name(0))
uid = o.comm_unique_id()
p("uid", uid.shape, uid[:8].tolist())
h = o.comm_init(uid, 0, 1, 0)
p("init", h)
p("info", o.comm_info(h))
y = torch.arange(8, device="cuda", dtype=torch.float32)
o.comm_allreduce_(h, y, "sum")
p("allreduce enqueued")
o.comm_wait(h)
torch.cuda.synchronize()
p("allreduce", y.tolist())
o.comm_sync(h)
o.comm_destroy(h)
p("destroyed")
