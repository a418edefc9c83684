"""BCE - log(Dice) segmentation loss with the reference's exact semantics.

Parity target: reference ``utils/utils.py:9-25``:

    loss = BCELoss(mean)(p, t) - log(2 * sum(p * [t == 1]) / (sum(p) + sum([t == 1]) + 1e-15))

* the Dice term is *global over the whole local batch*, not per-sample;
* ``dice_weight`` only toggles the term (truthy), it never scales it (quirk A12, kept);
* BCE clamps ``log`` at -100 like ``torch.nn.BCELoss``; everything is computed in fp32.

``Loss`` works on probabilities (the reference model's output).  ``LogitLoss`` takes logits and
is what the fused HIP path computes (sigmoid folded in, numerically identical up to the clamp).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

EPS = 1e-15


def bce_dice_from_probs(p: torch.Tensor, t: torch.Tensor, dice: bool = True) -> torch.Tensor:
    p = p.float()
    t = t.float()
    loss = F.binary_cross_entropy(p, t)
    if dice:
        dt = (t == 1).float()
        inter = (p * dt).sum()
        union = p.sum() + dt.sum() + EPS
        loss = loss - torch.log(2 * inter / union)
    return loss


class Loss:
    """Drop-in for the reference ``Loss`` (utils/utils.py:9)."""

    def __init__(self, dice_weight=1):
        self.dice_weight = dice_weight

    def __call__(self, outputs, targets):
        return bce_dice_from_probs(outputs, targets, bool(self.dice_weight))


def dice_score(p: torch.Tensor, t: torch.Tensor, threshold: float = 0.5) -> torch.Tensor:
    """Hard Dice of the thresholded prediction (the "Dice parity" metric of BASELINE.json)."""
    pred = (p.float() > threshold).float()
    tt = (t.float() == 1).float()
    inter = (pred * tt).sum()
    return (2 * inter + 1e-6) / (pred.sum() + tt.sum() + 1e-6)
