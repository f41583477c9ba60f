"""Training-step semantics of ``LightningWrappedModel`` (``scripts/train_utils.py:26-64``)
without the Lightning runtime (not installed; its control plane is out of scope).

``training_step`` computes the reference loss
``100 * mean_b( mean_ij (C - C^)^2 / mean_ij C^2 )``; ``configure_optimizers``
builds the same AdamW(amsgrad) (``scripts/train_utils.py:38-43``).
"""
from __future__ import annotations

from argparse import Namespace
from typing import Any

import torch


def stiffness_loss(pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """``scripts/train_utils.py:52-60`` (per-graph means over every non-batch dim: [B, 6, 6]
    as the reference, or the 21-vector of the vanilla CGC benchmark)."""
    dims = tuple(range(1, target.dim()))
    mean_stiffness = target.pow(2).mean(dim=dims)
    per_graph = torch.nn.functional.mse_loss(pred, target, reduction="none").mean(dim=dims)
    return 100 * (per_graph / mean_stiffness).mean()


class LightningWrappedModel(torch.nn.Module):
    def __init__(self, model: Any, params: Namespace) -> None:
        super().__init__()
        if isinstance(params, dict):
            params = Namespace(**params)
        self.params = params
        self.model = model(params)

    def configure_optimizers(self):
        p = self.params
        return torch.optim.AdamW(self.model.parameters(), lr=p.lr, betas=(p.beta1, 0.999),
                                 eps=p.epsilon, amsgrad=p.amsgrad, weight_decay=p.weight_decay)

    def training_step(self, batch, batch_idx: int = 0) -> torch.Tensor:
        out = self.model(batch)
        return stiffness_loss(out["stiffness"], batch["stiffness"])

    def predict_step(self, batch, batch_idx: int = 0):
        return self.model(batch), batch
