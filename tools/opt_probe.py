"""Time the flat Adam kernel on the headline's 72.2M-parameter buffers (one process per knob
setting: VINF_OPT_NT / VINF_OPT_BLOCKS are read once by the launcher)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vi_normflows_amd.ops._ext import native  # noqa: E402

native()
n = 72_200_000
dev = torch.device("cuda:0")
p, g, m, v = (torch.randn(n, device=dev) * 0.01 for _ in range(4))
v.abs_()
pbf = torch.empty(n, device=dev, dtype=torch.bfloat16)
step = torch.tensor(3.0, device=dev)
for _ in range(5):
    torch.ops.vinf.flat_optimizer(0, p, g, m, v, pbf, 1e-4, 0.9, 0.999, 1e-8, 0.0, step, 1.0, None, 1.0, None)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    torch.ops.vinf.flat_optimizer(0, p, g, m, v, pbf, 1e-4, 0.9, 0.999, 1e-8, 0.0, step, 1.0, None, 1.0, None)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1000 / 20
print(json.dumps({"nt": os.environ.get("VINF_OPT_NT", "0"), "blocks": os.environ.get("VINF_OPT_BLOCKS", "2048"),
                  "us": round(us, 1), "TBps": round(n * 30 / us / 1e6, 2)}))
