"""Carvana-layout folder dataset (reference utils/dataloading.py:12-78) on real image files: a tiny
``train_hq/*.jpg`` + ``train_masks/*_mask.gif`` tree written with PIL, then the dataset contract
(ids, resize semantics, value ranges, 0/255 mask normalisation, error cases) and one CPU training
epoch of ``train.py -t singleGPU --data-dir`` over it."""
import numpy as np
import pytest
import torch

from distributedpytorch_amd.data import BasicDataset, CarvanaDataset

PIL = pytest.importorskip("PIL")
from PIL import Image  # noqa: E402


def _write_tree(root, n=6, w=48, h=32, seed=0):
    rng = np.random.default_rng(seed)
    imgs, masks = root / "train_hq", root / "train_masks"
    imgs.mkdir(parents=True)
    masks.mkdir(parents=True)
    for i in range(n):
        rgb = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
        m = np.zeros((h, w), np.uint8)
        m[h // 4:3 * h // 4, w // 4 + i:3 * w // 4] = 255          # a car-shaped box, 0/255 like Carvana
        Image.fromarray(rgb).save(imgs / f"car{i:02d}.jpg", quality=95)
        Image.fromarray(m).save(masks / f"car{i:02d}_mask.gif")
    (imgs / ".DS_Store").write_bytes(b"")                        # hidden files are skipped
    return imgs, masks


def test_carvana_folder_items(tmp_path):
    imgs, masks = _write_tree(tmp_path)
    ds = CarvanaDataset(imgs, masks, newsize=(24, 16))
    assert len(ds) == 6 and ds.ids == [f"car{i:02d}" for i in range(6)]
    it = ds[2]
    assert it["image"].dtype == torch.float32 and tuple(it["image"].shape) == (3, 16, 24)
    assert 0.0 <= it["image"].min().item() and it["image"].max().item() <= 1.0
    assert it["mask"].dtype == torch.int64 and tuple(it["mask"].shape) == (16, 24)
    assert set(it["mask"].unique().tolist()) == {0, 1}                # 0/255 GIF -> {0, 1}
    # NEAREST resize of the mask: the box covers the middle half of the rows
    assert it["mask"][8, 12].item() == 1 and it["mask"][0, 0].item() == 0
    # BICUBIC resize of the image, HWC -> CHW, /255
    ref = np.asarray(Image.open(imgs / "car02.jpg").resize((24, 16), resample=Image.BICUBIC)).transpose(2, 0, 1) / 255.0
    assert np.allclose(it["image"].numpy(), ref, atol=1e-6)


def test_folder_errors(tmp_path):
    imgs, masks = _write_tree(tmp_path, n=3)
    with pytest.raises(RuntimeError, match="No input file found"):
        BasicDataset(tmp_path / "nowhere", masks)
    (masks / "car01_mask.gif").unlink()
    with pytest.raises(AssertionError, match="no mask or multiple masks"):
        CarvanaDataset(imgs, masks)
    Image.fromarray(np.zeros((10, 10), np.uint8)).save(masks / "car01_mask.gif")
    ds = CarvanaDataset(imgs, masks, newsize=(8, 8))
    with pytest.raises(AssertionError, match="should be the same size"):
        ds[1]


def test_npy_images_load_without_pickle(tmp_path):
    imgs, masks = tmp_path / "i", tmp_path / "m"
    imgs.mkdir()
    masks.mkdir()
    np.save(imgs / "a.npy", np.full((8, 8, 3), 128, np.uint8))
    np.save(masks / "a.npy", np.eye(8, dtype=np.uint8))
    it = BasicDataset(imgs, masks, newsize=(8, 8))[0]
    assert torch.allclose(it["image"], torch.full((3, 8, 8), 128 / 255.0, dtype=torch.float32))
    assert torch.equal(it["mask"], torch.eye(8, dtype=torch.int64))


def test_train_on_carvana_folder(tmp_path):
    """One CPU epoch of the reference single-GPU method over real files (-v: validation split)."""
    from distributedpytorch_amd.config import parse_args
    from distributedpytorch_amd.trainer import train
    _write_tree(tmp_path / "data", n=8)
    out = train(parse_args(["-e", "1", "-b", "2", "-v", "25", "--data-dir", str(tmp_path / "data"),
                            "--img-size", "32", "--model", "unet-tiny", "--backend", "torch", "--dtype", "fp32",
                            "--out-dir", str(tmp_path / "out"), "--log-every", "1"]))
    assert out["step"] == 3                                    # 6 train images / batch 2
    assert out["curves"].train and all(np.isfinite(r[2]) for r in out["curves"].train)
    assert out["curves"].val and np.isfinite(out["curves"].val[-1][2])
    assert (tmp_path / "out" / "checkpoints" / "singleGPU.pth").exists()
