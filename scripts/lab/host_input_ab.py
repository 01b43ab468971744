"""Lab: device-resident vs host-input pipeline steps timed alternately in one process, with the
host-side enqueue time of each run() (is the second pipeline host-bound?)."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "satellite-pose-estimation_amd"))
import torch  # noqa: E402

from spe.config import SpeConfig  # noqa: E402
from spe.models import DETR  # noqa: E402
from spe.pipeline import PosePipeline  # noqa: E402
from spe.solver import build_solver  # noqa: E402
from spe.synthetic import bench_images, fixed_bench_weights  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--rounds", type=int, default=3)
a = ap.parse_args()
dev = torch.device("cuda", 0)
cfg = SpeConfig()
w, _ = fixed_bench_weights(cfg, 0)
m = DETR(cfg, dtype="bf16")
m.load_state_dict(w)
solver = build_solver(argparse.Namespace(solver="epnp", repro=20))
B = 64
pool = bench_images(cfg, 0, 2 * B)
kw = dict(overlap=True, overlap_decode=True, overlap_backbone=True)
dp = PosePipeline(m, solver, B, device=dev, **kw)
dp.load(torch.from_numpy(pool["images"][:B]).to(dev), torch.from_numpy(pool["clip_bbox"][:B]).float().to(dev),
        torch.from_numpy(pool["quat"][:B]).to(dev), torch.from_numpy(pool["tvec"][:B]).to(dev))
hp = PosePipeline(m, solver, B, device=dev, host_input=True, **kw)
hp.load_host(torch.from_numpy(pool["crops_u8"]), torch.from_numpy(pool["clip_bbox"]),
             torch.from_numpy(pool["quat"]), torch.from_numpy(pool["tvec"]))


def timed(p, name):
    for _ in range(3):
        p.run()
    torch.cuda.synchronize()
    enq = 0.0
    t0 = time.perf_counter()
    for _ in range(a.steps):
        e0 = time.perf_counter()
        p.run()
        enq += time.perf_counter() - e0
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{name:6s} {1e3 * dt / a.steps:7.3f} ms/step  enqueue {1e3 * enq / a.steps:6.3f} ms/step", flush=True)


for r in range(a.rounds):
    timed(dp, "device")
    timed(hp, "host")
