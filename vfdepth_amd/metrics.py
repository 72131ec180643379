"""Depth metrics (the "Abs.Rel parity" half of BASELINE.json's metric).

`cal_depth_error` follows `/root/reference/utils/misc.py:85-98`; `compute_depth_losses` follows
`Logger.compute_depth_losses` (`/root/reference/utils/logger.py:193-247`): per camera, the
predicted depth is resized to the GT resolution (bilinear, align_corners=False), clamped to the
eval range, masked by GT range x camera mask, evaluated raw ("metric") and median-scaled
("median"), and averaged over cameras.  Results stay on the device until the final host copy.
"""
from collections import defaultdict

import torch
import torch.nn.functional as F

METRIC_NAMES = ['abs_rel', 'sq_rel', 'rms', 'log_rms', 'a1', 'a2', 'a3']   # logger.py:76 _metric_names


def cal_depth_error(pred, target):
    """abs_rel, sq_rel, rmse, rmse_log, a1, a2, a3 of flat depth tensors (misc.py:85-98)."""
    diff = pred - target
    abs_rel = torch.mean(torch.abs(diff) / target)
    sq_rel = torch.mean(diff.pow(2) / target)
    rmse = torch.sqrt(torch.mean(diff.pow(2)))
    rmse_log = torch.sqrt(torch.mean((torch.log(target) - torch.log(pred)).pow(2)))
    thresh = torch.max(target / pred, pred / target)
    return (abs_rel, sq_rel, rmse, rmse_log, (thresh < 1.25).float().mean(),
            (thresh < 1.25 ** 2).float().mean(), (thresh < 1.25 ** 3).float().mean())


def compute_depth_losses(inputs, outputs, num_cams, min_depth, max_depth, return_scales=False):
    """Per-camera depth errors averaged over cameras -> (metric dict, median-scaled dict)
    [+ median scales].  inputs['depth'] [B,N,1,h,w], inputs['mask'] [B,N,1,h,w],
    outputs[('cam',c)][('depth',0)] [B,1,H,W]."""
    metric, median = defaultdict(float), defaultdict(float)
    scales = []
    for cam in range(num_cams):
        gt = inputs['depth'][:, cam]
        h, w = gt.shape[-2:]
        pred = outputs[('cam', cam)][('depth', 0)].to(gt.device).detach()
        pred = torch.clamp(F.interpolate(pred, [h, w], mode='bilinear', align_corners=False), min_depth, max_depth)
        mask = ((gt > min_depth) * (gt < max_depth) * inputs['mask'][:, cam]).bool()
        gt, pred = gt[mask], pred[mask]
        scale = torch.median(gt) / torch.median(pred)
        scales.append(scale)
        em = cal_depth_error(torch.clamp(pred, min_depth, max_depth), gt)
        ed = cal_depth_error(torch.clamp(pred * scale, min_depth, max_depth), gt)
        for k, a, b in zip(METRIC_NAMES, em, ed):
            metric[k] += a
            median[k] += b
    metric = {k: v.cpu().numpy() / num_cams for k, v in metric.items()}
    median = {k: v.cpu().numpy() / num_cams for k, v in median.items()}
    if return_scales:
        return metric, median, [round(float(s), 2) for s in scales]
    return metric, median
