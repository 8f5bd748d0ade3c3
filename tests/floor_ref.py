"""Test-side torch form of the catalog-wide floor (search.union_floor runs only on the device,
as the ebt_union_floor kernel): the k-th largest of vals[r, b, j] - eps[r, b] over r and j."""
import torch


def union_floor_torch(vals: torch.Tensor, eps: torch.Tensor, k: int) -> torch.Tensor:
    R, B, kk = vals.shape
    lo = vals.double() - eps.double()[:, :, None]
    lo = torch.nan_to_num(lo, nan=float("-inf"), neginf=float("-inf"))
    lo = lo.permute(1, 0, 2).reshape(B, R * kk)
    return torch.topk(lo, k, dim=1).values[:, k - 1].contiguous()
