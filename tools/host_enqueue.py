"""Host enqueue time per forward vs GPU time per forward (cfg 2, B = 64): is the host ahead of the GPU?
usage: python3 tools/host_enqueue.py [iters]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sep_tfanet_vad_amd as pkg  # noqa: E402
from sep_tfanet_vad_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
cfg = pkg.CONFIG_WITH_VAD
net = pkg.SeparationModel(**cfg)
net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.make_state_dict(cfg, 1234).items()}, strict=True)
net = net.eval().to("cuda")
x = torch.from_numpy(synth.make_batch(64, 32000, 11)[0]).to("cuda")
with torch.no_grad():
    for _ in range(5):
        net(x)
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for _ in range(n):
        a = time.perf_counter()
        net(x)
        host.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
host.sort()
print(f"host enqueue per forward: median {host[n // 2] * 1e6:.1f} us, max {host[-1] * 1e6:.1f} us; "
      f"enqueue loop {(t1 - t0) / n * 1e6:.1f} us/forward; wall incl. drain {(t2 - t0) / n * 1e6:.1f} us/forward")
