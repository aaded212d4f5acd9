"""Probe: torch-ROCm's own GPU stack(...).mean(0) against the numpy
restatement oracle/torch_gpu_order.py, over many (N, M) shapes.  Prints one
JSON line per shape and a summary; used to pin the restatement before the
kernel mode is trusted (tests/test_gpu_torch_order.py is the committed test)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import torch_gpu_order as G  # noqa: E402

dev = torch.device("cuda", 0)
rng = np.random.default_rng(0)
bad = 0
shapes = [(n, m) for n in (2, 3, 4, 5, 7, 8, 9, 16, 17, 20, 24, 31, 32, 33, 40, 63, 64, 65, 100,
                           127, 128, 200, 300)
          for m in (1, 2, 3, 5, 6, 10, 16, 17, 64, 100, 432, 1000, 4096, 65536, 2359296)]
for n, m in shapes:
    if not G.supported(n, m) or n * m > 60_000_000:
        continue
    x = (rng.standard_normal((n, m)) * 10.0 ** rng.integers(-3, 4, (n, m))).astype(np.float32)
    rows = [torch.from_numpy(x[i]).to(dev) for i in range(n)]
    got = torch.stack(rows, 0).mean(0).cpu().numpy()
    want = G.gpu_mean0(x)
    mism = int((got.view(np.uint32) != want.view(np.uint32)).sum())
    bad += mism > 0
    print(json.dumps({"n": n, "m": m, "cfg": G.config(n, m), "mismatch": mism}), flush=True)
# int64 keys: .float() then the GPU mean, truncated into int64
for n in (2, 5, 20, 24, 33, 100):
    v = rng.integers(0, 3000, n)
    rows = [torch.tensor(int(a), device=dev).float() for a in v]
    got = torch.stack(rows, 0).mean(0)
    t = torch.zeros((), dtype=torch.int64, device=dev)
    t.copy_(got)
    want = G.gpu_mean_i64_trunc(v[:, None].astype(np.int64)).reshape(())
    ok = int(t.item()) == int(want)
    bad += not ok
    print(json.dumps({"n": n, "int64": True, "ok": ok}), flush=True)
print(json.dumps({"shapes_with_mismatch": bad}), flush=True)
