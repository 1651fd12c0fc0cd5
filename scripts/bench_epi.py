"""Epilogue-bound GEMMs (tiny K): how fast are the output/aux streams?"""
import sys
import torch
sys.path.insert(0, ".")
import ldnn  # noqa
from ldnn.ops import _ext
C = _ext.C()


def t(fn, it=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


M = N = 4096
for K in (16, 64):
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    wt = torch.randn(K, N, device="cuda").bfloat16()
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    aux = torch.randn(M, N, device="cuda").bfloat16()
    bias = torch.randn(N, device="cuda")
    for tile, direct in ((128, False), (256, True), (256, False)):
        us_f = t(lambda: C.gemm(x, w, y, True, True, C.EPI_BIAS_RELU, bias=bias, tile=tile, direct_epi=direct))
        us_d = t(lambda: C.gemm(x, wt, y, True, False, C.EPI_DRELU, aux=aux, tile=tile, direct_epi=direct))
        print(f"K={K} tile={tile} direct={direct}: fwd+bias+relu {us_f:.1f} us ({32e6/us_f/1e6:.2f} TB/s out), "
              f"dgrad+drelu {us_d:.1f} us ({64e6/us_d/1e6:.2f} TB/s out+aux)")
    us_t = t(lambda: torch.matmul(x, w.t()))
    print(f"K={K} torch matmul {us_t:.1f} us")
