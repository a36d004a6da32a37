"""ORACLE (test infrastructure only) -- integer/index work of SwinV2 in numpy.

Restates, without torch, the index semantics the HIP W-MSA kernels fold into
their address math.  Every table here must match the reference bit-exactly
(goldens: tests/golden/index_golden.npz, made by tests/golden/make_golden.py
from /root/reference/swinv2.py).
"""
import numpy as np


def effective_window(res_h: int, res_w: int, window: int, shift: int):
    """Window clamp of SwinTransformerBlock.__init__ (swinv2.py:328-334):
    when the feature map is no larger than the window, use one window covering
    it and no shift."""
    if min(res_h, res_w) <= window:
        return min(res_h, res_w), 0
    assert 0 <= shift < window
    return window, shift


def block_shift(block_idx: int, window: int) -> int:
    """BasicLayer alternation (swinv2.py:559): even blocks W-MSA, odd SW-MSA."""
    return 0 if block_idx % 2 == 0 else window // 2


def relative_position_index(window: int) -> np.ndarray:
    """[N, N] int64, N = window^2 (swinv2.py:176-190).

    rpi[i, j] = (ih - jh + w - 1) * (2w - 1) + (iw - jw + w - 1)
    with (ih, iw) = divmod(i, w)."""
    w = window
    t = np.arange(w * w)
    ih, iw = t // w, t % w
    dh = ih[:, None] - ih[None, :] + (w - 1)
    dw = iw[:, None] - iw[None, :] + (w - 1)
    return (dh * (2 * w - 1) + dw).astype(np.int64)


def relative_coords_table(window: int, pretrained_window: int = 0) -> np.ndarray:
    """[1, 2w-1, 2w-1, 2] float32 log-spaced CPB inputs (swinv2.py:147-171).

    value = sign(t) * log2(|t| + 1) / log2(8), t = 8 * delta / (pw - 1)
    (pw = pretrained window if > 0 else the window)."""
    w = window
    d = np.arange(-(w - 1), w, dtype=np.float32)
    tab = np.stack(np.meshgrid(d, d, indexing="ij"), axis=-1)[None].astype(np.float32)
    denom = np.float32((pretrained_window if pretrained_window > 0 else w) - 1)
    tab = tab / denom
    tab = tab * np.float32(8.0)
    tab = np.sign(tab) * np.log2(np.abs(tab) + np.float32(1.0)) / np.float32(3.0)
    return tab.astype(np.float32)


def window_gather_map(res_h: int, res_w: int, window: int, shift: int) -> np.ndarray:
    """[nW, N] int32: token (h*W + w) of the UN-shifted image that lands at
    position t of window k after roll(-shift) + window_partition
    (swinv2.py:69-83, 399-412).  window_reverse + roll(+shift)
    (swinv2.py:86-102, 420-429) scatters back through the same map."""
    w, s = window, shift
    nwh, nww = res_h // w, res_w // w
    k = np.arange(nwh * nww)
    t = np.arange(w * w)
    wh, ww = (k // nww)[:, None], (k % nww)[:, None]
    th, tw = (t // w)[None, :], (t % w)[None, :]
    src_h = (wh * w + th + s) % res_h
    src_w = (ww * w + tw + s) % res_w
    return (src_h * res_w + src_w).astype(np.int32)


def shift_region_ids(res_h: int, res_w: int, window: int, shift: int) -> np.ndarray:
    """[H, W] int region label in the SHIFTED frame (swinv2.py:359-375)."""
    def band(n):
        r = np.zeros(n, np.int64)
        r[n - window: n - shift] = 1
        r[n - shift:] = 2
        return r
    return 3 * band(res_h)[:, None] + band(res_w)[None, :]


def shift_mask(res_h: int, res_w: int, window: int, shift: int) -> np.ndarray:
    """[nW, N, N] float32 with 0 / -100 (swinv2.py:357-388); None if no shift."""
    if shift == 0:
        return None
    w = window
    reg = shift_region_ids(res_h, res_w, w, shift)
    nwh, nww = res_h // w, res_w // w
    win = reg.reshape(nwh, w, nww, w).transpose(0, 2, 1, 3).reshape(nwh * nww, w * w)
    same = win[:, :, None] == win[:, None, :]
    return np.where(same, np.float32(0.0), np.float32(-100.0)).astype(np.float32)


def patch_merge_gather_map(res_h: int, res_w: int) -> np.ndarray:
    """[H/2 * W/2, 4] int32: source token for each merged token's four
    C-wide slots, in the reference concat order x0, x1, x2, x3 =
    (even h, even w), (odd h, even w), (even h, odd w), (odd h, odd w)
    (swinv2.py:484-491)."""
    oh, ow = np.meshgrid(np.arange(res_h // 2), np.arange(res_w // 2), indexing="ij")
    oh, ow = oh.reshape(-1), ow.reshape(-1)
    dh = np.array([0, 1, 0, 1])
    dw = np.array([0, 0, 1, 1])
    src = (2 * oh[:, None] + dh[None, :]) * res_w + (2 * ow[:, None] + dw[None, :])
    return src.astype(np.int32)
