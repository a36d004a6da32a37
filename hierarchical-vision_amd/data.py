"""Device-side input normalisation -- the data.py slice on the hot path.

The reference normalises each uint8 batch from pil_image_collate (data.py:36-76) on the
device with composer's NormalizationFn (data.py:130-136, :154-164 DataSpec device_transforms):
f32 (x - mean) / std with mean / std in the 0-255 scale (data.py:128-133).  Here that is one
HIP kernel (hvk_normalize_u8), or -- when the model's PatchEmbed takes it (fuse_into) -- no
separate pass at all: the normalisation runs inside the patch gather that feeds the patch-
embedding GEMM (hvk_patchify_u8_bf16), so the f32 image batch is never written.  composer's
NormalizationFn is third-party (mosaicml 0.13.1, not vendored): its arithmetic is restated
from the published source and pinned against torch's own sub_ / div_ (parity unpinned by the
reference, which has no tests).
"""
import torch

from . import ops


def channel_stats(data_cfg):
    """(mean, std) in the 0-255 scale, as build_dataspec scales them (data.py:128-133)."""
    mean, std = list(data_cfg.channel_mean), list(data_cfg.channel_std)
    if all(m < 1 for m in mean):
        mean = [m * 255 for m in mean]
    if all(s < 1 for s in std):
        std = [s * 255 for s in std]
    return mean, std


class NormalizationFn:
    """composer.datasets.utils.NormalizationFn surface: called on a (images, targets) batch,
    returns the batch with images normalised to f32 (uint8 CUDA images: hvk_normalize_u8)."""

    def __init__(self, mean, std, ignore_background=False):
        if ignore_background:
            raise NotImplementedError("ignore_background is a segmentation option (ADE20k)")
        self.mean = mean
        self.std = std
        self._dev = {}

    def _stats(self, device):
        if device not in self._dev:
            self._dev[device] = (torch.tensor(self.mean, dtype=torch.float32, device=device),
                                 torch.tensor(self.std, dtype=torch.float32, device=device))
        return self._dev[device]

    def __call__(self, batch):
        xs, ys = batch
        if xs.is_cuda and xs.dtype == torch.uint8:
            m, s = self._stats(xs.device)
            return ops.normalize_u8(xs, m, s), ys
        m, s = (t.view(1, -1, 1, 1) for t in self._stats(xs.device))
        return xs.float().sub_(m).div_(s), ys

    def fuse_into(self, model):
        """Move the normalisation into the model's PatchEmbed (uint8 batches then go straight to
        the model); False when the model has no such entry point (the trainer keeps calling
        this transform)."""
        net = getattr(model, "module", model)
        pe = getattr(net, "patch_embed", None)
        if pe is None or not hasattr(pe, "set_input_normalization"):
            return False
        pe.set_input_normalization(self.mean, self.std)
        return True
