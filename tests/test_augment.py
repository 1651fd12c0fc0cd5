"""AutoAugment(CIFAR10) / flip+crop / normalise input kernel (augment.hip) against its NumPy
reference (data/autoaugment.py), plus op-level sanity of the reference itself.
Reference transform: BAR/dataloader.py:14-21 (torchvision AutoAugment, CIFAR10 policy).
torchvision is not importable here: parity with it is unpinned; kernel == reference is pinned."""
import time

import numpy as np
import pytest
import torch

from ldnn.data import autoaugment as AA
from ldnn.data.datasets import ArrayDataset
from ldnn.data.loader import DeviceLoader, augment_native


def _imgs(n=64, c=3, h=32, w=32, seed=0):
    rng = np.random.default_rng(seed)
    x = rng.integers(0, 256, (n, c, h, w), dtype=np.uint8)
    x[0] = 7            # constant image (AutoContrast / Equalize degenerate cases)
    x[1, :, :16] = 0    # two-level image
    x[1, :, 16:] = 200
    return x


# ------------------------------------------------------------------ reference (CPU)
def test_policy_and_magnitude_tables():
    assert AA.NUM_POLICIES == 25 and len(AA.CIFAR10_POLICY) == 25
    m = AA.magnitude_table(32, 32)
    np.testing.assert_allclose(m[AA.OP["ShearX"]], np.linspace(0, 0.3, 10), rtol=1e-6)
    np.testing.assert_allclose(m[AA.OP["TranslateX"]], np.linspace(0, 150 / 331 * 32, 10), rtol=1e-6)
    np.testing.assert_allclose(m[AA.OP["Rotate"]], np.linspace(0, 30, 10), rtol=1e-6)
    np.testing.assert_allclose(m[AA.OP["Solarize"]], np.linspace(255, 0, 10), rtol=1e-6)
    assert list(m[AA.OP["Posterize"]]) == [8, 8, 7, 7, 6, 6, 5, 5, 4, 4]


def test_reference_op_identities():
    img = _imgs(4)[3]
    ap = AA.apply_op
    assert np.array_equal(ap(ap(img, "Invert", 0), "Invert", 0), img)
    assert np.array_equal(ap(img, "Posterize", 8), img)
    for op in ("ShearX", "ShearY", "TranslateX", "TranslateY", "Rotate", "Brightness", "Color", "Contrast", "Sharpness"):
        assert np.array_equal(ap(img, op, 0.0), img), op
    t = ap(img, "TranslateX", 3.0)
    assert np.array_equal(t[:, :, 3:], img[:, :, :-3]) and not t[:, :, :3].any()
    ac = ap(_imgs(4)[1], "AutoContrast", 0)
    assert ac.min() == 0 and ac.max() == 255
    assert np.array_equal(ap(_imgs(4)[0], "Equalize", 0), _imgs(4)[0])   # one level: step 0 -> unchanged
    assert np.array_equal(ap(img, "Solarize", 256.0), img) and np.array_equal(ap(img, "Solarize", 0.0), 255 - img)


def test_cpu_loader_reproducible_and_matches_reference():
    imgs = _imgs(40)
    ds = ArrayDataset(torch.from_numpy(imgs), torch.zeros(40, dtype=torch.long), 10, None, None, "t")
    mk = lambda: DeviceLoader(ds, np.arange(40), 16, "cpu", augment="autoaugment+flipcrop", seed=5)  # noqa: E731
    a, b = list(mk()), list(mk())
    for (xa, _), (xb, _) in zip(a, b):
        assert torch.equal(xa, xb)
    l = mk()
    e0, e1 = [x for x, _ in l], [x for x, _ in l]
    assert not torch.equal(e0[0], e1[0])          # new draws each epoch
    raw = AA.augment_reference(imgs, np.arange(16), AA.batch_seed(5, 0, 0), AA.MODE_AUTOAUGMENT | AA.MODE_FLIP_CROP)
    np.testing.assert_allclose(e0[0].numpy(), raw.astype(np.float32) / 255.0, atol=1e-6)


# ------------------------------------------------------------------ kernel (GPU)
def _run(imgs, idx, seed, mode, fixed=None, out_dtype=torch.float32):
    dev = torch.device("cuda")
    im = torch.from_numpy(imgs).to(dev)
    ix = torch.as_tensor(idx, dtype=torch.long, device=dev)
    C = imgs.shape[1]
    out = torch.empty(len(idx), *imgs.shape[1:], dtype=out_dtype, device=dev)
    augment_native(im, ix, out, torch.ones(C, device=dev), torch.zeros(C, device=dev), seed, mode, 4, fixed)
    torch.cuda.synchronize()
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(3, 32, 32), (1, 28, 28), (3, 20, 24)])
def test_kernel_every_op_matches_reference(shape):
    imgs = _imgs(48, *shape, seed=1)
    idx = np.arange(48)[::-1].copy()
    for op in range(len(AA.OPS)):
        for bn in ((1, 5, 9) if op < AA.OP["AutoContrast"] else (0,)):
            for sg in (0, 1):
                got = _run(imgs, idx, 3, 0, fixed=(op, bn, sg)).cpu().numpy()
                ref = AA.augment_reference(imgs, idx, 3, 0, fixed=(op, bn, sg)).astype(np.float32)
                bad = np.argwhere(got != ref)
                assert bad.size == 0, (AA.OPS[op], bn, sg, shape, bad[:5])


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [AA.MODE_AUTOAUGMENT, AA.MODE_FLIP_CROP, AA.MODE_AUTOAUGMENT | AA.MODE_FLIP_CROP])
def test_kernel_policy_draws_match_reference(mode):
    imgs = _imgs(300, seed=2)
    idx = np.random.default_rng(0).integers(0, 300, 512)
    seed = AA.batch_seed(11, 2, 7)
    got = _run(imgs, idx, seed, mode).cpu().numpy()
    ref = AA.augment_reference(imgs, idx, seed, mode).astype(np.float32)
    assert np.array_equal(got, ref)
    # every sub-policy fires in a batch this size
    pols = {AA.draws(seed, b)["policy"] for b in range(len(idx))}
    assert len(pols) == 25


@pytest.mark.gpu
def test_device_loader_native_normalise_and_throughput():
    n = 4096
    imgs = _imgs(n, seed=3)
    ds = ArrayDataset(torch.from_numpy(imgs), torch.randint(0, 10, (n,)), 10, (0.5, 0.4, 0.3), (0.2, 0.25, 0.3), "t")
    plain = DeviceLoader(ds, np.arange(n), 256, "cuda", dtype=torch.float32)
    assert plain._native
    x, _ = next(iter(plain))
    ref = (torch.from_numpy(imgs[:256]).float() / 255.0 - torch.tensor([0.5, 0.4, 0.3]).view(1, 3, 1, 1)) / \
        torch.tensor([0.2, 0.25, 0.3]).view(1, 3, 1, 1)
    torch.testing.assert_close(x.cpu(), ref, rtol=1e-5, atol=1e-5)
    aug = DeviceLoader(ds, np.arange(n), 16384 // 4, "cuda", dtype=torch.bfloat16, augment="autoaugment")
    xb, _ = next(iter(aug))
    seed = AA.batch_seed(0, 0, 0)
    raw = AA.augment_reference(imgs, np.arange(4096), seed, AA.MODE_AUTOAUGMENT).astype(np.float32) / 255.0
    refn = (torch.from_numpy(raw) - torch.tensor([0.5, 0.4, 0.3]).view(1, 3, 1, 1)) / torch.tensor(
        [0.2, 0.25, 0.3]).view(1, 3, 1, 1)
    torch.testing.assert_close(xb.float().cpu(), refn, rtol=1e-2, atol=2e-2)
    # throughput: 16384 CIFAR images per launch
    big = torch.from_numpy(np.random.default_rng(4).integers(0, 256, (16384, 3, 32, 32), dtype=np.uint8)).cuda()
    ix = torch.randperm(16384, device="cuda")
    out = torch.empty(16384, 3, 32, 32, dtype=torch.bfloat16, device="cuda")
    a, b = torch.ones(3, device="cuda"), torch.zeros(3, device="cuda")
    for _ in range(3):
        augment_native(big, ix, out, a, b, 1, AA.MODE_AUTOAUGMENT | AA.MODE_FLIP_CROP)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(20):
        augment_native(big, ix, out, a, b, i, AA.MODE_AUTOAUGMENT | AA.MODE_FLIP_CROP)
    torch.cuda.synchronize()
    rate = 20 * 16384 / (time.perf_counter() - t0)
    print(f"augment throughput {rate / 1e6:.1f} M img/s")
    assert rate > 1e6
