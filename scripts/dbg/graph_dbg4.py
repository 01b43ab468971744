import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "satellite-pose-estimation_amd"))
import numpy as np, torch
from spe.config import SpeConfig
from spe.synthetic import random_weights, synthetic_batch
from spe.models import DETR
dev = torch.device("cuda:0")
cfg = SpeConfig(input_size=128, num_queries=11, enc_layers=2, dec_layers=2)
m = DETR(cfg, dtype="fp32"); m.load_state_dict(random_weights(cfg, 5))
B = 8
b = synthetic_batch(cfg, B, 700)
img = torch.from_numpy(b["images"]).to(dev); clip = torch.from_numpy(b["clip_bbox"]).float().to(dev)
ws = m.new_workspace(B, dev)
m.encode(img, ws)
def segs(a, b):
    d = (a != b).nonzero().flatten().cpu().numpy()
    if d.size == 0: return []
    br = np.nonzero(np.diff(d) > 64)[0]
    st = np.r_[d[0], d[br + 1]]; en = np.r_[d[br], d[-1]]
    return [(int(x), int(y)) for x, y in zip(st, en)]
ref = m.decode(B, ws, clip_bbox=clip)["pred_logits"].clone(); torch.cuda.synchronize()
e1 = ws.clone()
ref2 = m.decode(B, ws, clip_bbox=clip)["pred_logits"].clone(); torch.cuda.synchronize()
print("eager twice", (ref2 - ref).abs().max().item(), segs(ws, e1))
s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    out = m.decode(B, ws, clip_bbox=clip)
torch.cuda.synchronize()
print("after capture", segs(ws, e1))
snaps = []
for r in range(3):
    g.replay(); torch.cuda.synchronize()
    print("replay", r, (out["pred_logits"] - ref).abs().max().item(), segs(ws, e1), flush=True)
