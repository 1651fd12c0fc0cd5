"""Run the bandwidth-bound kernels of the headline step at its shapes (batch 16384,
hidden 4096): the fused dReLU/bias-grad pass and the SGD update, 5 launches each,
for rocprofv3 counter passes (scripts/pmc_membound.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ldnn  # noqa: E402,F401
from ldnn.ops import _ext  # noqa: E402

C = _ext.C()
B, H, P = 16384, 4096, 20037642
dz = torch.randn(B, H, device="cuda").bfloat16()
h = torch.randn(B, H, device="cuda").relu().bfloat16()
db = torch.zeros(H, device="cuda")
p, g, m = (torch.randn(P, device="cuda") for _ in range(3))
sh = torch.empty(P, dtype=torch.bfloat16, device="cuda")
hp = torch.tensor([0.01, 0.0], device="cuda")
for _ in range(5):
    C.act_bwd_colsum(dz, h, dz, db, C.ACT_RELU, True)
    C.sgd_step(p, g, m, sh, hp, 1.0, 0.9, 0.0, 0.0, False, False)
torch.cuda.synchronize()
print("ok")
