#!/bin/bash
# space-to-depth stem wgrad: tests, stem wgrad micro, step A/B
set -o pipefail
O=gpurun_out/r3s2s2d
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_layers_gpu.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -80 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 120 python -u - > $O/micro.txt 2>&1 <<'PY' || { tail -20 $O/micro.txt; exit 1; }
import torch, json, sys
sys.path.insert(0, ".")
import ldnn
from ldnn.ops import _ext
C = _ext.C()
for N in (64, 256):
    x = torch.zeros(N, 224, 224, 8, device="cuda", dtype=torch.bfloat16); x[..., :3] = torch.randn(N, 224, 224, 3, device="cuda").bfloat16()
    gy = torch.randn(N, 112, 112, 64, device="cuda").bfloat16()
    dw = torch.empty(64, 7, 7, 8, device="cuda")
    for mode in (0, 1):
        C.set_conv_stem_s2d(mode)
        for _ in range(3): C.conv_wgrad(gy, x, dw, 2, 3, 0.0, real_channels=3)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(); s.record()
        for _ in range(20): C.conv_wgrad(gy, x, dw, 2, 3, 0.0, real_channels=3)
        e.record(); torch.cuda.synchronize()
        print(json.dumps({"N": N, "stem_s2d": mode, "wgrad_us": round(s.elapsed_time(e) / 20 * 1e3, 2)}), flush=True)
    C.set_conv_stem_s2d(1)
PY
grep -v amdgpu.ids $O/micro.txt
rm -f gpurun_out/ab_cnn.jsonl
bash scripts/ab_cnn.sh "resnet18:64 resnet18:256" "LDNN_CONV_STEM_S2D=0" "LDNN_CONV_STEM_S2D=1" > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
