"""Folder datasets in the Carvana layout (reference ``utils/dataloading.py:12-78``).

Behaviour kept: ids = image file stems (hidden files skipped), ``RuntimeError`` when the image
dir is empty, exactly one image and one mask per id, BICUBIC resize for images / NEAREST for
masks to ``newsize=(W, H)``, HWC->CHW, /255, items ``{'image': f32[C,H,W], 'mask': i64[H,W]}``.

Changes: ``.npy/.npz`` load with ``allow_pickle=False`` and ``.pt/.pth`` with
``weights_only=True`` (never unpickle data files); the file glob is done once at construction
instead of per item.  Binary masks stored as 0/255 are normalised to 0/1 (the reference's loss
raises on 0/255 targets).
"""
from __future__ import annotations

import logging
import os
from pathlib import Path

import numpy as np
import torch
from torch.utils.data import Dataset


def _load_image(path: Path):
    from PIL import Image

    ext = path.suffix.lower()
    if ext in (".npy",):
        return Image.fromarray(np.load(path, allow_pickle=False))
    if ext in (".npz",):
        with np.load(path, allow_pickle=False) as z:
            return Image.fromarray(z[z.files[0]])
    if ext in (".pt", ".pth"):
        return Image.fromarray(torch.load(path, weights_only=True).numpy())
    return Image.open(path)


class BasicDataset(Dataset):
    def __init__(self, images_dir, masks_dir, newsize=(960, 640), mask_suffix: str = ""):
        self.images_dir = Path(images_dir)
        self.masks_dir = Path(masks_dir)
        self.newsize = (int(newsize[0]), int(newsize[1]))
        assert self.newsize[0] > 0 and self.newsize[1] > 0, "newsize must be positive"
        self.mask_suffix = mask_suffix
        files = sorted(f for f in os.listdir(self.images_dir) if not f.startswith(".")) \
            if self.images_dir.is_dir() else []
        self.ids = [os.path.splitext(f)[0] for f in files]
        if not self.ids:
            raise RuntimeError(f"No input file found in {images_dir}, make sure you put your images there")
        masks = {}
        for f in os.listdir(self.masks_dir):
            masks.setdefault(os.path.splitext(f)[0], []).append(self.masks_dir / f)
        imgs = {}
        for f in files:
            imgs.setdefault(os.path.splitext(f)[0], []).append(self.images_dir / f)
        self._pairs = []
        for name in self.ids:
            m = masks.get(name + mask_suffix, [])
            i = imgs.get(name, [])
            assert len(m) == 1, f"Either no mask or multiple masks found for the ID {name}: {m}"
            assert len(i) == 1, f"Either no image or multiple images found for the ID {name}: {i}"
            self._pairs.append((i[0], m[0]))
        logging.info(f"Creating dataset with {len(self.ids)} examples")

    def __len__(self):
        return len(self.ids)

    @staticmethod
    def preprocess(pil_img, newsize, is_mask):
        from PIL import Image

        new_w, new_h = newsize
        pil_img = pil_img.resize((new_w, new_h), resample=Image.NEAREST if is_mask else Image.BICUBIC)
        arr = np.asarray(pil_img)
        if is_mask:
            if arr.ndim == 3:
                arr = arr[..., 0]
            if arr.max(initial=0) > 1:
                arr = (arr > 127).astype(np.int64)
            return arr
        if arr.ndim == 2:
            arr = arr[np.newaxis, ...]
        else:
            arr = arr.transpose((2, 0, 1))
        return arr / 255.0

    def __getitem__(self, idx):
        img_path, mask_path = self._pairs[idx]
        img = _load_image(img_path)
        mask = _load_image(mask_path)
        assert img.size == mask.size, \
            f"Image and mask {self.ids[idx]} should be the same size, but are {img.size} and {mask.size}"
        img = self.preprocess(img, self.newsize, is_mask=False)
        mask = self.preprocess(mask, self.newsize, is_mask=True)
        return {
            "image": torch.as_tensor(img.copy()).float().contiguous(),
            "mask": torch.as_tensor(mask.copy()).long().contiguous(),
        }


class CarvanaDataset(BasicDataset):
    def __init__(self, images_dir, masks_dir, newsize=(960, 640)):
        super().__init__(images_dir, masks_dir, newsize, mask_suffix="_mask")
