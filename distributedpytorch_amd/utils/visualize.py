"""Image / mask plotting (reference ``utils/utils.py:38-51`` ``plot_img_and_mask``, unused there).

Same layout: the input image, then one panel per mask class.  ``path`` saves the figure instead
of showing it (headless nodes); matplotlib is imported lazily so training never depends on it.
"""
from __future__ import annotations


def plot_img_and_mask(img, mask, path: str = None):
    import matplotlib
    if path is not None:
        matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    import numpy as np

    img = np.asarray(img)
    if img.ndim == 3 and img.shape[0] in (1, 3):   # CHW tensor -> HWC
        img = img.transpose(1, 2, 0)
    mask = np.asarray(mask)
    classes = mask.shape[0] if mask.ndim > 2 else 1
    fig, ax = plt.subplots(1, classes + 1)
    ax[0].set_title("Input image")
    ax[0].imshow(img)
    if classes > 1:
        for i in range(classes):
            ax[i + 1].set_title(f"Output mask (class {i + 1})")
            ax[i + 1].imshow(mask[i])
    else:
        ax[1].set_title("Output mask")
        ax[1].imshow(mask)
    for a in ax:
        a.set_xticks([])
        a.set_yticks([])
    if path is not None:
        fig.savefig(path, bbox_inches="tight")
        plt.close(fig)
    else:
        plt.show()
    return fig
