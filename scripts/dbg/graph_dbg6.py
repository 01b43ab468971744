import sys, os, time
if len(sys.argv) > 1 and sys.argv[1] == "pre":
    os.environ["DEBUG_CLR_GRAPH_PACKET_CAPTURE"] = "0"
import torch
if len(sys.argv) > 1 and sys.argv[1] == "post":
    os.environ["DEBUG_CLR_GRAPH_PACKET_CAPTURE"] = "0"
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
ref = m(img, clip_bbox=clip)["pred_logits"].clone()
s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    m(img, clip_bbox=clip)
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    o = m(img, clip_bbox=clip)
res = []
for tag, pre in (("b2b", None), ("sync", "sync"), ("sleep", "sleep"), ("b2b2", None), ("sync2", "sync")):
    if pre == "sync": torch.cuda.synchronize()
    if pre == "sleep": time.sleep(0.3)
    g.replay()
    res.append((tag, o["pred_logits"].clone()))
torch.cuda.synchronize()
print(os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE"), [(t, (x - ref).abs().max().item()) for t, x in res], flush=True)
