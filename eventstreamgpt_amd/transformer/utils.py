"""Loss reductions (``EventStream/transformer/utils.py:134-234``), PyTorch form for API compatibility.
The training path evaluates them inside the fused loss kernel."""
import torch


def safe_weighted_avg(X: torch.Tensor, weights: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    torch._assert((weights >= 0).all(), "weights should be >= 0")
    shape_err = (f"weights {weights.shape} must be the same shape as X {X.shape} "
                 "or the same shape as X excluding the second to last dimension")
    if len(weights.shape) < len(X.shape):
        try:
            weights = weights.unsqueeze(-2).expand_as(X)
        except RuntimeError as e:
            raise AssertionError(shape_err) from e
    else:
        torch._assert(weights.shape == X.shape, shape_err)
    w = weights.float()
    denom = w.sum(dim=-1)
    safe = torch.where(denom > 0, denom, torch.ones_like(denom))
    return torch.where(denom > 0, (X * w).sum(dim=-1) / safe, torch.zeros_like(denom)), denom


def weighted_loss(loss_per_event: torch.Tensor, event_mask: torch.Tensor) -> torch.Tensor:
    per_subject, n = safe_weighted_avg(loss_per_event, event_mask)
    return safe_weighted_avg(per_subject, n > 0)[0]
