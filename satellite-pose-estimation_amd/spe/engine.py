"""evaluate() with the reference's signature (REV/engine.py:78-135).

Per batch: one device pass (model + fused PostProcess), one batched solver launch and one
D2H copy of the pose records, instead of the reference's per-image Python solver loop.
The criterion (Hungarian matcher + losses, REV/engine.py:99-112) runs on the device
(spe.models.SetCriterion) when given; its losses are logged like the reference's
MetricLogger: per-batch values averaged over batches, weighted ("loss", "loss_ce", ...) and
"<k>_unscaled", plus "class_error".
"""
from __future__ import annotations

import torch

from . import _lib
from . import dist as spe_dist
from .speed_eval import SpeedEval, device_speed_score


@torch.no_grad()
def evaluate(model, criterion, postprocessors, data_loader, gt_file, solver, device, output_dir=None):
    evaluator = SpeedEval(gt_file, solver)
    ceres = getattr(solver, "mode", None) == _lib.SPE_PNP_EPNP_CERES
    if ceres:
        # EPnPCeresSolver's per-image thresholds come from the ground-truth box areas: refuse up front a
        # ground truth without them (load_ground_truth sets "area" only from bbox_xxyy).  The area-driven
        # threshold itself is parity unpinned: the REV SpeedEval calls the solver without an area
        # (REV/datasets/speed.py:399, commented out); UNC's passes it (speed_dataset.py:396-399).
        missing = [f for f, g in evaluator.ground_truth.items() if "area" not in g]
        if missing:
            raise ValueError(f"EPnPCeresSolver evaluation needs ground-truth box areas (bbox_xxyy); "
                             f"{len(missing)} entries lack them, e.g. {missing[0]}")
    meters = {}

    def log(k, v):
        s = meters.setdefault(k, [0.0, 0])
        s[0] += float(v)
        s[1] += 1

    for samples, targets in data_loader:
        samples = samples.to(device)
        filenames = [t["filename"] for t in targets]
        clip = torch.stack([torch.as_tensor(t["clip_bbox"], dtype=torch.float32) for t in targets]).to(device)
        outputs = model(samples, clip_bbox=clip)
        if criterion is not None:
            ld = criterion(outputs, [{k: v.to(device) for k, v in t.items() if torch.is_tensor(v)} for t in targets])
            ld = {k: float(v) for k, v in ld.items()}
            if spe_dist.is_dist():                            # utils.reduce_dict (REV/engine.py:103)
                vals = torch.tensor([ld[k] for k in sorted(ld)], dtype=torch.float64, device=device)
                torch.distributed.all_reduce(vals)
                ld = dict(zip(sorted(ld), (vals / torch.distributed.get_world_size()).tolist()))
            wd = criterion.weight_dict
            scaled = {k: v * wd[k] for k, v in ld.items() if k in wd}
            log("loss", sum(scaled.values()))
            for k, v in scaled.items():
                log(k, v)
            for k, v in ld.items():
                log(k + "_unscaled", v)
            log("class_error", ld["class_error"])
        gt = [evaluator.ground_truth[f] for f in filenames]
        if ceres:
            # EPnPCeresSolver: one threshold per image from its ground-truth box area (UNC SpeedEval
            # passes ground_truth[filename]["area"], src/data/speed/speed_dataset.py:396-399)
            poses = solver.solve_batch(outputs["points_px"], outputs["probs"], outputs.get("sigmas"),
                                       area=[g["area"] for g in gt])
        else:
            poses = solver.solve_batch(outputs["points_px"], outputs["probs"], outputs.get("sigmas"))
        q_gt = torch.tensor([g["quat"] for g in gt], dtype=torch.float64, device=device)
        t_gt = torch.tensor([g["tvec"] for g in gt], dtype=torch.float64, device=device)
        s_t, s_q = device_speed_score(poses["quat"], poses["tvec"], q_gt, t_gt)
        sig = outputs.get("sigmas")
        assess = solver.self_assess(outputs["probs"], sig, poses) if sig is not None else None
        evaluator.update_batch(filenames, outputs["points_px"], outputs["probs"], poses, s_t, s_q, sig, assess)
    evaluator.log = spe_dist.all_gather_log(evaluator.log)
    evaluator.summarize()
    stats = {k: s / max(n, 1) for k, (s, n) in meters.items()}
    stats["speed_eval_pose"] = evaluator.stats
    return stats, evaluator
