"""Batched solver latency per mode on the solver stress set (tests/helpers.solver_stress_set):
one launch of spe_pnp_batch per mode at B images, HIP-event timed.
usage: python scripts/solver_bench.py [--batch 32] [--iters 5]"""
import argparse
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "satellite-pose-estimation_amd"), os.path.join(REPO, "tests")]
from helpers import solver_stress_set  # noqa: E402
from spe.solver import PoseSolver  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    pts, probs, q, t, sig = solver_stress_set(a.batch, seed=5)
    P, R, S = (torch.from_numpy(x).to(dev) for x in (pts, probs, sig))
    for mode, name in [(0, "epnp"), (3, "epnp_lm"), (1, "ransac_p3p_lm"), (2, "epnp_ransac_sigma")]:
        s = PoseSolver(mode=mode, repro=25.0 if mode == 2 else 20.0)
        sg = S if mode == 2 else None
        out = s.solve_batch(P, R, sg)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            s.solve_batch(P, R, sg, out=out)
        e1.record()
        torch.cuda.synchronize()
        st = out["status"].cpu().numpy()
        print(f"{name:18s} B={a.batch}: {e0.elapsed_time(e1) / a.iters:.3f} ms/launch  status={np.bincount(st, minlength=5).tolist()}")


if __name__ == "__main__":
    main()
