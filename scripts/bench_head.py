"""Head kernel timing: fwd+xent alone vs with the fused dgrad (LDNN_HEAD_DBG selects
debug cut-downs of the fused path)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ldnn  # noqa: E402,F401
from ldnn.ops import _ext  # noqa: E402
from scripts.bench_wgrad import timeit  # noqa: E402

C = _ext.C()
B, H, NC = 4096, 4096, 16
h = torch.randn(B, H, device="cuda").relu().bfloat16()
W = (torch.randn(NC, H, device="cuda") * 0.02).bfloat16()
bias = torch.zeros(NC, device="cuda")
y = torch.randint(0, 10, (B,), device="cuda")
lg, dl = torch.empty(B, NC, device="cuda", dtype=torch.bfloat16), torch.empty(B, NC, device="cuda", dtype=torch.bfloat16)
st = torch.zeros(B // 16, 2, device="cuda")
dh = torch.empty(B, H, device="cuda", dtype=torch.bfloat16)
db = torch.zeros(H, device="cuda")
ws = torch.empty(C.head_dgrad_ws_floats(B, H), device="cuda")
tag = os.environ.get("LDNN_HEAD_DBG", "0")
print("dbg", tag, "fwd only us", round(timeit(lambda: C.head_fwd_xent(h, W, bias, y, lg, dl, st, 10, 1.0 / B)), 2))
print("dbg", tag, "fused us", round(timeit(lambda: C.head_fwd_xent(h, W, bias, y, lg, dl, st, 10, 1.0 / B, dh=dh, dbias=db,
                                                                   dgrad_epi=C.EPI_DRELU, dbias_ws=ws)), 2))
print("dbg", tag, "fused no dbias us", round(timeit(lambda: C.head_fwd_xent(h, W, bias, y, lg, dl, st, 10, 1.0 / B, dh=dh,
                                                                            dgrad_epi=C.EPI_DRELU)), 2))
