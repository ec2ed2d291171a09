"""Probe: can RCCL run a 2-rank group whose ranks share one GPU?  (Used to
decide whether the 2-rank all-gather can be exercised on a one-GPU box.)
  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29561 tools/probes/rccl_two_ranks_one_gpu.py
"""
import json
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
out = {"rank": rank, "world": world}
try:
    dist.init_process_group("nccl", device_id=dev)
    x = torch.full((4,), rank + 1, dtype=torch.int32, device=dev)
    ys = [torch.empty_like(x) for _ in range(world)]
    dist.all_gather(ys, x)
    torch.cuda.synchronize()
    out["gathered"] = [int(y[0].item()) for y in ys]
    out["ok"] = out["gathered"] == list(range(1, world + 1))
    dist.destroy_process_group()
except Exception as e:  # noqa: BLE001
    out["ok"] = False
    out["error"] = f"{type(e).__name__}: {e}"[:400]
print(json.dumps(out), flush=True)
