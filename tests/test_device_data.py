"""HBM-resident synthetic dataset (data/device.py): same items as the CPU dataset (masks exact,
images up to the pixel-noise realisation), deterministic per index, batches gathered through
``random_split`` subsets with the same samplers as the host loaders.  Runs on any device; the
trainer uses it on the GPU (no DataLoader / H2D on the hot path)."""
import torch

from distributedpytorch_amd.data import SyntheticSegmentation, split_dataset
from distributedpytorch_amd.data.device import DeviceSyntheticSegmentation, device_loaders


def test_device_items_match_cpu_dataset():
    cpu = SyntheticSegmentation(6, (40, 24), 3, seed=9)
    dev = DeviceSyntheticSegmentation(6, (40, 24), 3, seed=9, device="cpu", chunk=4)
    for i in range(6):
        a, b = cpu[i], dev[i]
        assert torch.equal(a["mask"], b["mask"])
        assert b["image"].dtype == torch.float32 and b["image"].shape == (3, 40, 24)
        # only the +/-0.05 noise and the uint8 (k/255) storage differ
        assert (a["image"] - b["image"]).abs().max() <= 0.1 + 0.5 / 255 + 1e-6
        assert 0.0 <= float(b["image"].min()) and float(b["image"].max()) <= 1.0
    again = DeviceSyntheticSegmentation(6, (40, 24), 3, seed=9, device="cpu", chunk=6)
    assert torch.equal(again.images, dev.images)                          # independent of chunking


def test_device_loader_batches_follow_sampler_and_split():
    ds = DeviceSyntheticSegmentation(20, (16, 16), 3, seed=1, device="cpu")
    tr, va = split_dataset(ds, 25, seed=0)
    tl, vl, sampler = device_loaders(tr, va, 4, seed=3)
    sampler.set_epoch(1)
    order = list(iter(sampler))
    seen = []
    for k, (img, tgt) in enumerate(tl):
        nb = img.shape[0]
        assert img.shape == (nb, 3, 16, 16) and tgt.shape == (nb, 1, 16, 16) and tgt.dtype == torch.float32
        for j in range(nb):
            base = tr.indices[order[4 * k + j]]
            assert torch.equal(img[j], ds.to_float(ds.images[base])) and torch.equal(tgt[j, 0], ds.masks[base].float())
            seen.append(base)
    assert sorted(seen) == sorted(tr.indices) and len(tl) == 4
    assert sum(x.shape[0] for x, _ in vl) == len(va) == 5
