"""Time spe_pnp_batch per solver mode on the tests' stress set (device-resident inputs, HIP
events around N repeated solves).  Usage: python scripts/solver_bench.py [B] [Q]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "satellite-pose-estimation_amd"), os.path.join(ROOT, "tests")]
from helpers import solver_stress_set  # noqa: E402
from spe.solver import PoseSolver  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
Q = int(sys.argv[2]) if len(sys.argv) > 2 else 11
dev = torch.device("cuda:0")
pts, probs, q, t, sig = solver_stress_set(B, seed=3, Q=Q)
P, R, S = (torch.from_numpy(x).to(dev) for x in (pts, probs, sig))
for mode, name in [(0, "epnp"), (3, "epnp_lm"), (1, "ransac_p3p_lm"), (2, "epnp_ransac_sigma")]:
    s = PoseSolver(mode=mode, repro=25.0 if mode == 2 else 20.0)
    sg = S if mode == 2 else None
    o = s.solve_batch(P, R, sg)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 10
    e0.record()
    for _ in range(n):
        s.solve_batch(P, R, sg, out=o)
    e1.record()
    torch.cuda.synchronize()
    st = torch.bincount(o["status"].long(), minlength=5).tolist()
    print(f"{name:18s} B={B} Q={Q}: {e0.elapsed_time(e1) / n:.3f} ms/solve  status={st}", flush=True)
