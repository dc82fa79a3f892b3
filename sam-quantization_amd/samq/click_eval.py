"""Click-simulation mask IoU: the reference's 5-click evaluation loop.

Restates ``script/evaluation2.py``: ``get_iou`` (``:156-167``, with ``ignore_label``),
``get_next_click_torch`` (``:170-200``: a click drawn uniformly from the false-negative OR
false-positive pixels of the previous prediction, positive iff it is a false negative) and the
per-image loop of ``main`` (``:226-381``: clicks accumulate, the previous low-res logits are fed
back as the mask prompt from the second click on, ``multimask_output=False``, IoU of the
upsampled mask against the ground truth after every click; the image's score is the IoU after
the last click).  The reference draws clicks with the global ``np.random``; here an explicit
``numpy.random.Generator`` keeps a run reproducible (pass the same seed to compare two encoders).

Inputs are the image embedding(s) from any encoder (the HIP engine, the oracle, a reference
golden) and ground-truth masks ``(B, 1, H, W)`` with 1 = object, 0 = background and
``ignore_label`` (-1) for pixels that count for neither.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch
import torch.nn.functional as F


def get_iou(gt_mask: torch.Tensor, pred_mask: torch.Tensor, ignore_label: int = -1) -> torch.Tensor:
    """IoU of ``pred_mask`` with the object pixels of ``gt_mask``, ignored pixels excluded from both
    intersection and union (reference ``evaluation2.py:156-167``; summed over the whole batch)."""
    keep = gt_mask != ignore_label
    obj = gt_mask == 1
    pred = pred_mask.bool()
    inter = torch.logical_and(torch.logical_and(pred, obj), keep).sum()
    union = torch.logical_and(torch.logical_or(pred, obj), keep).sum()
    return inter / union


def get_next_click_torch(prev_seg: torch.Tensor, gt_semantic_seg: torch.Tensor,
                         rng: Optional[np.random.Generator] = None):
    """One click per image (reference ``evaluation2.py:170-200``): uniform over the error pixels of
    ``prev_seg > 0`` vs ``gt > 0``; returns lists of (1, 1, 2) xy points and (1, 1) labels."""
    pred = prev_seg > 0
    true = gt_semantic_seg > 0
    fn = torch.logical_and(true, torch.logical_not(pred))
    fp = torch.logical_and(torch.logical_not(true), pred)
    err = torch.logical_or(fn, fp)
    pts, lbls = [], []
    for i in range(gt_semantic_seg.shape[0]):
        cand = torch.argwhere(err[i])                     # (n, 3): channel, y, x
        j = (rng.integers(len(cand)) if rng is not None else np.random.randint(len(cand)))
        p = cand[j]
        pos = bool(fn[i, 0, p[1], p[2]])
        pts.append(torch.tensor([int(p[2]), int(p[1])]).reshape(1, 1, 2))
        lbls.append(torch.tensor([int(pos)]).reshape(1, 1))
    return pts, lbls


@torch.no_grad()
def click_iou(prompt_encoder, mask_decoder, image_embedding: torch.Tensor, gt_masks: torch.Tensor,
              num_clicks: int = 5, seed: int = 0, ignore_label: int = -1, clicks=None,
              return_trace: bool = False):
    """The reference's click loop for ONE image embedding ``(1, 256, 64, 64)`` and ``gt_masks``
    ``(B, 1, H, W)`` (B objects of that image, each its own episode).  Returns the IoU after every
    click for each object: ``[[iou_click1, ..., iou_clickN], ...]``.

    ``clicks`` (from an earlier call's trace) replays that click sequence instead of sampling it:
    the same (point, label) prompts with this embedding's own low-res logits fed back, so two
    encoders can be compared mask by mask along one episode.  ``return_trace=True`` returns
    ``(ious, trace)`` with ``trace[b] = {"clicks": [(xy, label), ...], "masks": [bool (H, W), ...]}``."""
    dev = image_embedding.device
    rng = np.random.Generator(np.random.PCG64(seed))
    out, trace = [], []
    for b in range(gt_masks.shape[0]):
        gt = gt_masks[b:b + 1].to(dev)
        prev = torch.zeros_like(gt, dtype=torch.float32)
        pts, lbls, low, ious = [], [], None, []
        tr = {"clicks": [], "masks": []}
        for k in range(num_clicks):
            if clicks is None:
                p, lab = get_next_click_torch(prev, gt, rng)
                p, lab = torch.cat(p), torch.cat(lab)
            else:
                xy, lv = clicks[b]["clicks"][k]
                p, lab = torch.tensor([[xy]]), torch.tensor([[lv]])
            tr["clicks"].append(((int(p[0, 0, 0]), int(p[0, 0, 1])), int(lab[0, 0])))
            pts.append(p.to(dev).float())
            lbls.append(lab.to(dev))
            sparse, dense = prompt_encoder(points=(torch.cat(pts, 1), torch.cat(lbls, 1)), boxes=None,
                                           masks=None if k == 0 else low)
            low, _ = mask_decoder(image_embedding.float(), prompt_encoder.get_dense_pe(), sparse, dense, False)
            prev = F.interpolate(low, size=gt.shape[-2:], mode="bilinear", align_corners=False)
            ious.append(float(get_iou(gt, prev > 0, ignore_label)))
            if return_trace:
                tr["masks"].append((prev > 0)[0, 0].cpu())
        out.append(ious)
        trace.append(tr)
    return (out, trace) if return_trace else out


def synthetic_gt_masks(n: int, size: int = 1024, seed: int = 0, ignore_band: int = 6) -> torch.Tensor:
    """``n`` seeded elliptical objects ``(n, 1, size, size)`` (1 inside, 0 outside) with an
    ``ignore_label`` (-1) band of ``ignore_band`` pixels on the boundary, the way SBD marks
    uncertain object borders (the evaluation data itself is not available offline)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    yy, xx = np.mgrid[0:size, 0:size].astype(np.float32)
    masks = np.zeros((n, 1, size, size), np.float32)
    for i in range(n):
        cy, cx = rng.uniform(0.3, 0.7, 2) * size
        ry, rx = rng.uniform(0.08, 0.25, 2) * size
        th = rng.uniform(0, np.pi)
        c, s = np.cos(th), np.sin(th)
        u = ((xx - cx) * c + (yy - cy) * s) / rx
        v = (-(xx - cx) * s + (yy - cy) * c) / ry
        r = np.sqrt(u * u + v * v)
        band = ignore_band / min(rx, ry)
        m = (r <= 1.0).astype(np.float32)
        m[np.abs(r - 1.0) < band] = -1.0
        masks[i, 0] = m
    return torch.from_numpy(masks)
