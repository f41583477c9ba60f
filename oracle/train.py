"""Loss of ``LightningWrappedModel.training_step`` (``scripts/train_utils.py:45-64``).

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).
"""
import torch


def stiffness_loss(pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """``100 * mean_b( mean_ij (C-C^)^2 / mean_ij C^2 )`` (``scripts/train_utils.py:54-60``)."""
    mean_stiffness = target.pow(2).mean(dim=(1, 2))
    per_graph = torch.nn.functional.mse_loss(pred, target, reduction="none").mean(dim=(1, 2))
    return 100 * (per_graph / mean_stiffness).mean()
