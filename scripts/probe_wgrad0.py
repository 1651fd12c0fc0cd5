import sys, torch
sys.path.insert(0, ".")
import ldnn
from ldnn.ops import _ext
C = _ext.C()
def t(fn, it=10):
    fn(); torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(it): fn()
        e1.record(); torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / it * 1e3)
    return round(best, 1)
for (M, N, K) in ((4096, 784, 4096), (4096, 784, 16384), (4096, 1024, 4096), (4096, 768, 4096), (4096, 4096, 4096)):
    dz = torch.randn(K, M, device="cuda").bfloat16(); h = torch.randn(K, N, device="cuda").bfloat16()
    dW = torch.empty(M, N, device="cuda")
    r = {"MNK": (M, N, K), "sk1": t(lambda: C.gemm(dz, h, dW, False, False, tile=256, variant=32))}
    for sk in (2, 4):
        ne, nc = C.gemm_pp_ws(M, N, sk); ws = torch.empty(ne, device="cuda"); cnt = torch.zeros(nc, device="cuda", dtype=torch.int32)
        r[f"sk{sk}"] = t(lambda: C.gemm(dz, h, dW, False, False, tile=256, variant=32, splitk=sk, ws=ws, cnt=cnt))
    r["lib"] = t(lambda: torch.mm(dz.t(), h, out_dtype=torch.float32, out=dW))
    print(r, flush=True)
