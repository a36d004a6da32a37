"""ORACLE (test infrastructure only) -- functional fp32 CPU restatement of the
SwinV2 forward in swinv2.py, driven by a flat state dict whose key names are
those of the reference module tree (swinv2.py:673-845).

It deliberately does NOT share code or structure with the product: windows
are formed with the numpy gather maps of ``index_ref`` instead of
roll + view/permute, so it doubles as an independent check of the product's
index math.  It also serves as the timed CPU baseline in bench.py (kind
"port").
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from . import index_ref

LOGIT_CLAMP_MAX = float(torch.log(torch.tensor(1.0 / 0.01)))  # swinv2.py:138


def model_geometry(img_size=224, patch_size=4, embed_dim=96, depths=(2, 2, 6, 2),
                   num_heads=(3, 6, 12, 24), window_size=7,
                   pretrained_window_sizes=(0, 0, 0, 0)):
    """Per-block (res, C, nH, window, shift, pretrained window) list,
    following SwinTransformerV2.__init__ / BasicLayer (swinv2.py:757-779,
    552-572) and the window clamp (swinv2.py:328-331)."""
    res = img_size // patch_size
    stages = []
    for i, d in enumerate(depths):
        r = res // (2 ** i)
        blocks = []
        for j in range(d):
            w, s = index_ref.effective_window(r, r, window_size,
                                              index_ref.block_shift(j, window_size))
            blocks.append(dict(res=r, dim=embed_dim * 2 ** i, heads=num_heads[i],
                               window=w, shift=s, pw=pretrained_window_sizes[i]))
        stages.append(dict(res=r, dim=embed_dim * 2 ** i, blocks=blocks,
                           merge=i < len(depths) - 1))
    return stages


def cpb_bias(p, pre, window, pw, heads):
    """16 * sigmoid(cpb_mlp(relative_coords_table))[rpi] -> [nH, N, N]
    (swinv2.py:141-145, 233-246)."""
    tab = torch.from_numpy(index_ref.relative_coords_table(window, pw)).reshape(-1, 2)
    hid = F.relu(tab @ p[pre + "cpb_mlp.0.weight"].T + p[pre + "cpb_mlp.0.bias"])
    out = hid @ p[pre + "cpb_mlp.2.weight"].T  # [(2w-1)^2, nH]
    rpi = torch.from_numpy(index_ref.relative_position_index(window)).reshape(-1)
    n = window * window
    bias = out[rpi].reshape(n, n, heads).permute(2, 0, 1)
    return 16.0 * torch.sigmoid(bias)


def window_attention(p, pre, xw, heads, window, pw, mask):
    """WindowAttention.forward (swinv2.py:204-264) on windows xw [B_, N, C]."""
    bw, n, c = xw.shape
    d = c // heads
    qkv_b = torch.cat([p[pre + "q_bias"], torch.zeros_like(p[pre + "v_bias"]),
                       p[pre + "v_bias"]])
    qkv = (xw @ p[pre + "qkv.weight"].T + qkv_b).reshape(bw, n, 3, heads, d)
    q, k, v = (qkv[:, :, i].transpose(1, 2) for i in range(3))  # [B_, nH, N, d]
    qn = q / q.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    kn = k / k.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    scale = torch.clamp(p[pre + "logit_scale"], max=LOGIT_CLAMP_MAX).exp()  # [nH,1,1]
    s = (qn @ kn.transpose(-1, -2)) * scale
    s = s + cpb_bias(p, pre, window, pw, heads)[None]
    if mask is not None:
        nw = mask.shape[0]
        s = (s.reshape(bw // nw, nw, heads, n, n) + mask[None, :, None]).reshape(bw, heads, n, n)
    a = torch.softmax(s, dim=-1)
    o = (a @ v).transpose(1, 2).reshape(bw, n, c)
    return o @ p[pre + "proj.weight"].T + p[pre + "proj.bias"]


def swin_block(p, pre, x, blk):
    """SwinTransformerBlock.forward (swinv2.py:390-436), res-post-norm."""
    b, L, c = x.shape
    r, w, s = blk["res"], blk["window"], blk["shift"]
    gmap = torch.from_numpy(index_ref.window_gather_map(r, r, w, s).astype(np.int64))
    nw, n = gmap.shape
    xw = x[:, gmap.reshape(-1)].reshape(b * nw, n, c)
    m = index_ref.shift_mask(r, r, w, s)
    mask = torch.from_numpy(m) if m is not None else None
    aw = window_attention(p, pre + "attn.", xw, blk["heads"], w, blk["pw"], mask)
    a = torch.empty_like(x)
    a[:, gmap.reshape(-1)] = aw.reshape(b, nw * n, c)
    x = x + F.layer_norm(a, (c,), p[pre + "norm1.weight"], p[pre + "norm1.bias"], 1e-5)
    h = F.gelu(x @ p[pre + "mlp.fc1.weight"].T + p[pre + "mlp.fc1.bias"])
    h = h @ p[pre + "mlp.fc2.weight"].T + p[pre + "mlp.fc2.bias"]
    return x + F.layer_norm(h, (c,), p[pre + "norm2.weight"], p[pre + "norm2.bias"], 1e-5)


def patch_merging(p, pre, x, res):
    """PatchMerging.forward (swinv2.py:475-496)."""
    b, L, c = x.shape
    g = torch.from_numpy(index_ref.patch_merge_gather_map(res, res).astype(np.int64))
    xm = x[:, g.reshape(-1)].reshape(b, g.shape[0], 4 * c)
    y = xm @ p[pre + "reduction.weight"].T
    return F.layer_norm(y, (2 * c,), p[pre + "norm.weight"], p[pre + "norm.bias"], 1e-5)


def forward_features(p, x, geom, patch_size=4):
    """PatchEmbed + stages + final LN + avgpool (swinv2.py:648-657, 818-840)."""
    y = F.conv2d(x, p["patch_embed.proj.weight"], p["patch_embed.proj.bias"],
                 stride=patch_size)
    b, c = y.shape[:2]
    y = y.reshape(b, c, -1).transpose(1, 2)
    y = F.layer_norm(y, (c,), p["patch_embed.norm.weight"], p["patch_embed.norm.bias"], 1e-5)
    for i, st in enumerate(geom):
        for j, blk in enumerate(st["blocks"]):
            y = swin_block(p, f"layers.{i}.blocks.{j}.", y, blk)
        if st["merge"]:
            y = patch_merging(p, f"layers.{i}.downsample.", y, st["res"])
    c = y.shape[-1]
    y = F.layer_norm(y, (c,), p["norm.weight"], p["norm.bias"], 1e-5)
    return y.mean(dim=1)


def forward(p, x, geom, patch_size=4):
    """SwinTransformerV2.forward (swinv2.py:842-845): flat head or the list of
    MultitaskHead logits (swinv2.py:36-40)."""
    f = forward_features(p, x, geom, patch_size)
    if "head.weight" in p:
        return f @ p["head.weight"].T + p["head.bias"]
    outs, i = [], 0
    while f"head.heads.{i}.weight" in p:
        outs.append(f @ p[f"head.heads.{i}.weight"].T + p[f"head.heads.{i}.bias"])
        i += 1
    return outs


def flops_per_image(geom, num_classes=1000, patch_res=56, embed_dim=96, in_chans=3,
                    patch_size=4):
    """MAC count, same accounting as SwinTransformerV2.flops (swinv2.py:847-867)."""
    f = patch_res * patch_res * embed_dim * in_chans * patch_size * patch_size
    f += patch_res * patch_res * embed_dim
    for st in geom:
        for blk in st["blocks"]:
            r, c, w = blk["res"], blk["dim"], blk["window"]
            n = w * w
            nw = r * r / (w * w)
            f += 2 * c * r * r
            f += nw * (n * c * 3 * c + 2 * n * n * c + n * c * c)
            f += 2 * r * r * c * c * 4
        if st["merge"]:
            r, c = st["res"], st["dim"]
            f += (r // 2) * (r // 2) * 4 * c * 2 * c + r * r * c // 2
    nf = geom[-1]["dim"]
    f += nf * patch_res * patch_res // (2 ** len(geom))
    f += nf * (num_classes if isinstance(num_classes, int) else sum(num_classes))
    return f


def init_params_from_rng(state_shapes: dict, seed: int) -> dict:
    """Deterministic parameter draw shared by the golden generator and the
    tests: per key, numpy default_rng(seed + crc32(key)), with scales chosen
    so that every sub-path is exercised -- post-norm gammas are NOT zero
    (SURVEY.md §0 finding 5)."""
    import zlib
    out = {}
    for name in sorted(state_shapes):
        shape = tuple(state_shapes[name])
        rng = np.random.default_rng(seed + zlib.crc32(name.encode()))
        if name.endswith("logit_scale"):
            v = np.log(10.0) + 0.3 * rng.standard_normal(shape)
        elif "norm" in name and name.endswith("weight"):
            v = 1.0 + 0.2 * rng.standard_normal(shape)
        elif "norm" in name and name.endswith("bias"):
            v = 0.1 * rng.standard_normal(shape)
        elif "cpb_mlp.0" in name:
            v = 0.5 * rng.standard_normal(shape)
        elif "cpb_mlp.2" in name:
            v = 0.1 * rng.standard_normal(shape)
        elif name.endswith("bias"):
            v = 0.02 * rng.standard_normal(shape)
        else:
            fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else shape[0]
            v = rng.standard_normal(shape) / math.sqrt(fan_in)
        out[name] = torch.from_numpy(np.asarray(v, np.float32))
    return out


def state_shapes(img_size=224, patch_size=4, in_chans=3, embed_dim=96, depths=(2, 2, 6, 2),
                 num_heads=(3, 6, 12, 24), window_size=7, num_classes=1000, mlp_ratio=4.0,
                 pretrained_window_sizes=(0, 0, 0, 0)):
    """Learnable-parameter key -> shape of the reference module tree
    (swinv2.py:192-200, 336-355, 472-473, 640-645, 781-795, 141-145)."""
    s = {"patch_embed.proj.weight": (embed_dim, in_chans, patch_size, patch_size),
         "patch_embed.proj.bias": (embed_dim,),
         "patch_embed.norm.weight": (embed_dim,), "patch_embed.norm.bias": (embed_dim,)}
    for i, d in enumerate(depths):
        c, h = embed_dim * 2 ** i, num_heads[i]
        for j in range(d):
            p = f"layers.{i}.blocks.{j}."
            hid = int(c * mlp_ratio)
            s.update({p + "norm1.weight": (c,), p + "norm1.bias": (c,),
                      p + "attn.logit_scale": (h, 1, 1), p + "attn.q_bias": (c,),
                      p + "attn.v_bias": (c,), p + "attn.cpb_mlp.0.weight": (512, 2),
                      p + "attn.cpb_mlp.0.bias": (512,), p + "attn.cpb_mlp.2.weight": (h, 512),
                      p + "attn.qkv.weight": (3 * c, c), p + "attn.proj.weight": (c, c),
                      p + "attn.proj.bias": (c,), p + "norm2.weight": (c,),
                      p + "norm2.bias": (c,), p + "mlp.fc1.weight": (hid, c),
                      p + "mlp.fc1.bias": (hid,), p + "mlp.fc2.weight": (c, hid),
                      p + "mlp.fc2.bias": (c,)})
        if i < len(depths) - 1:
            p = f"layers.{i}.downsample."
            s.update({p + "reduction.weight": (2 * c, 4 * c), p + "norm.weight": (2 * c,),
                      p + "norm.bias": (2 * c,)})
    nf = embed_dim * 2 ** (len(depths) - 1)
    s.update({"norm.weight": (nf,), "norm.bias": (nf,)})
    if isinstance(num_classes, int):
        s.update({"head.weight": (num_classes, nf), "head.bias": (num_classes,)})
    else:
        for i, n in enumerate(num_classes):
            s.update({f"head.heads.{i}.weight": (n, nf), f"head.heads.{i}.bias": (n,)})
    return s


def wmsa_core_ref(qkv, bias_table, scale, H, W, heads, window, shift):
    """Attention core from the qkv projection to the pre-proj output, on
    UN-partitioned tokens: qkv [B, H*W, 3C] -> [B, H*W, C] (fp32, CPU).
    Restates swinv2.py:221-261 with the roll/partition of 399-412 and the
    reverse of 420-429.  bias_table [heads, (2w-1)^2] = 16*sigmoid(cpb);
    scale [heads] = exp(clamp(logit_scale))."""
    b, L, c3 = qkv.shape
    c = c3 // 3
    d = c // heads
    g = torch.from_numpy(index_ref.window_gather_map(H, W, window, shift).astype(np.int64))
    nw, n = g.shape
    qw = qkv[:, g.reshape(-1)].reshape(b * nw, n, 3, heads, d)
    q, k, v = (qw[:, :, i].transpose(1, 2) for i in range(3))
    qn = q / q.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    kn = k / k.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    s = (qn @ kn.transpose(-1, -2)) * scale.reshape(1, heads, 1, 1)
    rpi = torch.from_numpy(index_ref.relative_position_index(window)).reshape(-1)
    s = s + bias_table[:, rpi].reshape(1, heads, n, n)
    m = index_ref.shift_mask(H, W, window, shift)
    if m is not None:
        s = (s.reshape(b, nw, heads, n, n) + torch.from_numpy(m)[None, :, None]).reshape(b * nw, heads, n, n)
    o = (torch.softmax(s, dim=-1) @ v).transpose(1, 2).reshape(b, nw * n, c)
    out = torch.empty(b, L, c, dtype=o.dtype)
    out[:, g.reshape(-1)] = o
    return out
