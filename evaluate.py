#!/usr/bin/env python3
"""Validation loop, API- and CLI-compatible with the reference ``evaluate.py:6-25``.

``evaluate(model, dataloader, criterion) -> float`` is the reference function (mean per-batch loss,
model put back in train mode); it also works for the framework's strategies through
:func:`distributedpytorch_amd.trainer.evaluate` (sharded, loss + Dice).  As a script it scores a
checkpoint:

    python evaluate.py -c singleGPU --synthetic --img-size 512 -b 8 [--backend hip]
"""
import argparse
import os

import numpy as np
import torch


def evaluate(model, dataloader, criterion, device=None):
    """Reference semantics: mean over validation batches of ``criterion(model(images), masks)``."""
    device = device or next(model.parameters()).device
    model.eval()
    losses = []
    with torch.no_grad():
        for batch in dataloader:
            if isinstance(batch, dict):
                images, masks = batch["image"], batch["mask"]
            else:
                images, masks = batch
            images = images.to(device, torch.float32)
            true_masks = masks.to(device, torch.float32)
            if true_masks.dim() == 3:
                true_masks = true_masks.unsqueeze(1)
            losses.append(float(criterion(model(images), true_masks)))
    model.train()
    return float(np.mean(losses)) if losses else float("nan")


def main(argv=None):
    from distributedpytorch_amd.config import TrainConfig
    from distributedpytorch_amd.data import SyntheticSegmentation, CarvanaDataset, build_loaders, split_dataset
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.trainer import SingleDevice, evaluate as evaluate_strategy
    from distributedpytorch_amd.utils import load_model_state

    ap = argparse.ArgumentParser(description="Evaluate a UNet checkpoint (val loss + Dice)")
    ap.add_argument("--checkpoint", "-c", default=None, help="checkpoints/<NAME>.pth")
    ap.add_argument("--load", "-l", default=None, help="explicit .pth path")
    ap.add_argument("--batch-size", "-b", type=int, default=4)
    ap.add_argument("--validation", "-v", type=float, default=10.0)
    ap.add_argument("--img-size", type=int, nargs="+", default=[640, 960])
    ap.add_argument("--synthetic", action="store_true")
    ap.add_argument("--synthetic-len", type=int, default=64)
    ap.add_argument("--data-dir", default="./data")
    ap.add_argument("--out-dir", default=".")
    ap.add_argument("--model", default="unet")
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"])
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp32"],
                    help="compute dtype (default bf16 on a GPU, fp32 on CPU; on a GPU fp32 runs the fp32 HIP engine)")
    ap.add_argument("--seed", "-s", type=int, default=42)
    a = ap.parse_args(argv)
    H, W = (a.img_size[0], a.img_size[-1])
    model = build_model(a.model)
    path = a.load or (os.path.join(a.out_dir, "checkpoints", f"{a.checkpoint}.pth") if a.checkpoint else None)
    if path:
        load_model_state(model, path)
    dev = "cuda:0" if torch.cuda.is_available() else "cpu"
    dtype = a.dtype or ("bf16" if dev != "cpu" else "fp32")
    cfg = TrainConfig(backend=a.backend, img_size=(H, W), dtype=dtype, synthetic=a.synthetic,
                      synthetic_len=a.synthetic_len, seed=a.seed, val=a.validation, data_dir=a.data_dir)
    strat = SingleDevice(cfg, model, dev)
    if a.synthetic and dev != "cpu":
        # the SAME validation images train.py --synthetic held out (GPU-resident set, seed, split)
        from distributedpytorch_amd.trainer import build_datasets
        from distributedpytorch_amd.data.device import device_loaders
        train_set, val_set = build_datasets(cfg, dev)
        _, val_loader, _ = device_loaders(train_set, val_set, a.batch_size)
    else:
        ds = SyntheticSegmentation(a.synthetic_len, (H, W), 3, seed=a.seed) if a.synthetic else \
            CarvanaDataset(os.path.join(a.data_dir, "train_hq"), os.path.join(a.data_dir, "train_masks"), newsize=(W, H))
        _, val_set = split_dataset(ds, a.validation, seed=0)
        _, val_loader, _ = build_loaders(val_set, val_set, a.batch_size)
    loss, dice = evaluate_strategy(strat, val_loader)
    print(f"backend {strat.compute.name} dtype {dtype}")
    print(f"val_loss {loss:.5f} dice {dice:.4f} ({len(val_set)} images, checkpoint {path})")
    return loss, dice


if __name__ == "__main__":
    main()
