"""RCCL (torch.distributed "nccl" on ROCm) on the GPU box: the collectives contact_zones_amd.parallel
issues once per run (broadcast, all_reduce, all_gather / all_gather_into_tensor, barrier) on device
tensors, in a one-rank process group.  A one-GPU box cannot hold two RCCL ranks (RCCL refuses two
ranks on one device), so the multi-rank logic is covered by the world_size-2 gloo tests
(tests/test_parallel.py); this checks that RCCL itself initialises and moves device data with this
image's environment (HSA_ENABLE_IPC_MODE_LEGACY=0), which the driver's 8-GPU runs rely on."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

SCRIPT = r"""
import json, torch, torch.distributed as dist
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", device_id=dev)
x = torch.arange(6, dtype=torch.float64, device=dev)
dist.all_reduce(x, op=dist.ReduceOp.MAX)
seed = torch.tensor([1234], dtype=torch.int64, device=dev)
dist.broadcast(seed, src=0)
out = torch.empty(6, dtype=torch.float64, device=dev)
dist.all_gather_into_tensor(out, x)
parts = [torch.empty(2, dtype=torch.float64, device=dev)]
dist.all_gather(parts, x[:2].contiguous())
box = [{"winner": 3}]
dist.broadcast_object_list(box, src=0, device=dev)
dist.barrier()
torch.cuda.synchronize()
print(json.dumps({"backend": dist.get_backend(), "x": x.tolist(), "seed": int(seed.item()),
                  "out": out.tolist(), "parts": parts[0].tolist(), "box": box[0]}))
dist.destroy_process_group()
"""


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_single_rank_collectives(gpu_available):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE="1",
               RANK="0", LOCAL_RANK="0")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, "-c", SCRIPT], capture_output=True, text=True, timeout=100, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    got = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert got["backend"] == "nccl"
    assert got["x"] == [0.0, 1.0, 2.0, 3.0, 4.0, 5.0]
    assert got["out"] == got["x"] and got["parts"] == [0.0, 1.0]
    assert got["seed"] == 1234 and got["box"] == {"winner": 3}
