"""Layer table of a UNet preset: output shape, parameters, forward GFLOP, activation bytes.

Counterpart of the reference's torchsummary dump ``model/modelsummary.txt``:
``python -m distributedpytorch_amd.models.summary [--model unet] [--hw 640 960] [--batch 1]``.
Computed analytically from the preset (no forward pass), so it works for any resolution.
"""
from __future__ import annotations

import argparse

from .unet import PRESETS, UNetConfig, build_model, count_params


def layer_table(cfg: UNetConfig, h: int, w: int, batch: int = 1, bytes_per_el: int = 4):
    rows = []

    def conv(name, cin, cout, H, W, k=3):
        params = cout * cin * k * k + cout
        rows.append((name, (batch, cout, H, W), params, 2.0 * H * W * cin * cout * k * k * batch / 1e9))

    H, W, cin = h, w, cfg.in_channels
    for i, wd in enumerate(cfg.widths):
        conv(f"encoder.conv{i + 1}.conv_block.0", cin, wd, H, W)
        conv(f"encoder.conv{i + 1}.conv_block.2", wd, wd, H, W)
        rows.append((f"encoder.maxpool (level {i + 1})", (batch, wd, H // 2, W // 2), 0, 0.0))
        H, W, cin = H // 2, W // 2, wd
    conv("mid.conv_block.0", cin, cfg.mid_width, H, W)
    conv("mid.conv_block.2", cfg.mid_width, cfg.mid_width, H, W)
    cin = cfg.mid_width
    for i, wd in enumerate(reversed(cfg.widths)):
        rows.append((f"decoder.deconv{i + 1}", (batch, wd, 2 * H, 2 * W), cin * wd * 4 + wd,
                     2.0 * H * W * cin * wd * 4 * batch / 1e9))
        H, W = 2 * H, 2 * W
        rows.append((f"decoder.cat{i + 1} (skip | up)", (batch, 2 * wd, H, W), 0, 0.0))
        conv(f"decoder.conv{i + 1}.conv_block.0", 2 * wd, wd, H, W)
        conv(f"decoder.conv{i + 1}.conv_block.2", wd, wd, H, W)
        cin = wd
    conv("segmap", cfg.base, cfg.out_channels, H, W, k=1)
    rows.append(("sigmoid", (batch, cfg.out_channels, H, W), 0, 0.0))
    return rows


def format_table(cfg: UNetConfig, h: int, w: int, batch: int = 1) -> str:
    rows = layer_table(cfg, h, w, batch)
    out = [f"{'Layer':<36}{'Output shape':>24}{'Param #':>12}{'GFLOP':>10}", "=" * 82]
    act = 0
    for name, shape, p, gf in rows:
        out.append(f"{name:<36}{str(list(shape)):>24}{p:>12,}{gf:>10.2f}")
        n = 1
        for d in shape:
            n *= d
        act += n
    params = sum(r[2] for r in rows)
    gf = sum(r[3] for r in rows)
    out += ["=" * 82, f"Total params: {params:,}", f"Forward GFLOP (batch {batch}): {gf:.2f}",
            f"Forward activations: {act * 4 / 2 ** 20:.2f} MB fp32 / {act * 2 / 2 ** 20:.2f} MB bf16",
            f"Params size: {params * 4 / 2 ** 20:.2f} MB fp32"]
    return "\n".join(out)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--model", default="unet", choices=sorted(PRESETS))
    ap.add_argument("--hw", type=int, nargs=2, default=[640, 960])
    ap.add_argument("--batch", type=int, default=1)
    a = ap.parse_args(argv)
    cfg = PRESETS[a.model]
    text = format_table(cfg, a.hw[0], a.hw[1], a.batch)
    assert count_params(build_model(a.model)) == sum(r[2] for r in layer_table(cfg, *a.hw))
    print(text)
    return text


if __name__ == "__main__":
    main()
