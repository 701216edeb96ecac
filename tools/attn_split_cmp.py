"""Cross-check of tools/attn_split_ab.py's saved gradients between settings (max abs difference / max abs value)."""
import sys

import torch

a = torch.load(sys.argv[1], weights_only=True)
worst = 0.0
for other in sys.argv[2:]:
    b = torch.load(other, weights_only=True)
    for k in a:
        d = (a[k] - b[k]).abs().max().item() / max(a[k].abs().max().item(), 1e-30)
        worst = max(worst, d)
        print(f"{other} {k}: {d:.3e}")
print("worst", worst)
assert worst < 2e-2, worst
