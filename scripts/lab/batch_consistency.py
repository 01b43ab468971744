"""bf16 forward at batch B vs the same first 64 images at batch 64: max |d pred_points|, label agreement.
    python scripts/lab/batch_consistency.py 64 128 192 256"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "satellite-pose-estimation_amd"))
from spe.config import SpeConfig  # noqa: E402
from spe.models import DETR  # noqa: E402
from spe.synthetic import bench_images, fixed_bench_weights  # noqa: E402

cfg = SpeConfig(input_size=416, num_queries=11, enc_layers=6, dec_layers=6)
w, _ = fixed_bench_weights(cfg, 0)
dev = torch.device("cuda", 0)
dt = os.environ.get("DT", "bf16")
m = DETR(cfg, dtype=dt)
m.load_state_dict(w)
data = bench_images(cfg, 0, 256)
x = torch.from_numpy(data["images"]).to(dev)
clip = torch.from_numpy(data["clip_bbox"]).float().to(dev)
ref = m(x[:64], clip_bbox=clip[:64], return_hs=True)
torch.cuda.synchronize()
rp, rl, rh = ref["pred_points"].clone(), ref["pred_logits"].argmax(-1).clone(), ref["hs"][-1].clone()
for B in [int(a) for a in sys.argv[1:]]:
    o = m(x[:B], clip_bbox=clip[:B], return_hs=True)
    torch.cuda.synchronize()
    d = (o["pred_points"][:64] - rp).abs().max().item()
    la = (o["pred_logits"][:64].argmax(-1) == rl).float().mean().item()
    dh = (o["hs"][-1][:64] - rh).abs().max().item()
    print(f"{dt} B={B}: max |d points| {d:.3e}  |d hs| {dh:.3e}  label agreement {la:.3f}", flush=True)
