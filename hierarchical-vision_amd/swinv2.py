"""SwinV2 for MI355X -- drop-in for the reference's swinv2.py.

Same class names, constructor signatures and state-dict keys as
/root/reference/swinv2.py (so official / reference checkpoints load), but the
block is re-planned around the hardware:

* The residual stream is carried as a ``ResidualStream`` (f32 master copy +
  bf16 copy that feeds the next GEMM), both written by one fused LayerNorm
  kernel -- the AMP reference keeps the same f32 residual (LayerNorm is an
  autocast-f32 op) but needs extra cast passes.
* qkv / proj are token-wise, so they run on UN-partitioned tokens; the
  cyclic shift, window partition, cosine attention, CPB bias, shift mask,
  softmax, P@V and window reverse are one HIP kernel (``ops.window_attention_core``)
  that addresses windows by index math.  torch.roll / window_partition /
  window_reverse (swinv2.py:69-102, 399-429) never materialise.
* Post-norm + DropPath + residual add is one kernel (``ops.layer_norm_residual``).
* PatchMerging's strided 2x2 gather rides in its reduction GEMM's operand loads both ways
  (``ops.merge_linear``; ``ops.patch_merge_gather`` + ``ops.linear`` where not built).
* Dense contractions (qkv, proj, fc1, fc2, reduction, patch embedding) run on
  libhvk's MFMA GEMMs in bf16 under autocast (``ops.linear``: the skinny
  weight-stationary kernel at the SwinV2-T stage 0-1 widths, the tiled kernel
  elsewhere, the weight-gradient kernel for every weight and bias gradient); only
  the classifier / multitask heads (M = batch) stay on hipBLASLt via torch.
"""
import dataclasses
import re
from typing import NamedTuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
import torch.utils.checkpoint as checkpoint

from . import ops
from .options import OPTIONS
from .hierarchy import MultitaskHead  # noqa: F401  (re-exported like swinv2.py:12-40)


def to_2tuple(x):
    return tuple(x) if isinstance(x, (list, tuple)) else (x, x)


class ResidualStream(NamedTuple):
    f32: torch.Tensor   # [B, L, C] float32 residual stream
    bf16: torch.Tensor  # [B, L, C] bfloat16 copy (GEMM operand)


def _as_stream(x):
    if isinstance(x, ResidualStream):
        return x
    return ResidualStream(x.float().contiguous(), x.to(torch.bfloat16).contiguous())


def _drop_path_scale(p, training, batch, device):
    """Per-sample DropPath factor (timm DropPath, scale_by_keep): 0 or 1/keep."""
    if p <= 0.0 or not training:
        return None
    keep = 1.0 - p
    return torch.empty(batch, device=device, dtype=torch.float32).bernoulli_(keep).div_(keep)


# --------------------------------------------------------------------------- index tables
def relative_coords_table(window, pretrained_window):
    """Log-spaced CPB inputs [1, 2w-1, 2w-1, 2] (swinv2.py:147-171)."""
    wh, ww = window
    dh = torch.arange(-(wh - 1), wh, dtype=torch.float32)
    dw = torch.arange(-(ww - 1), ww, dtype=torch.float32)
    t = torch.stack(torch.meshgrid(dh, dw, indexing="ij"), dim=-1).unsqueeze(0)
    den = pretrained_window if pretrained_window[0] > 0 else window
    t[..., 0] /= den[0] - 1
    t[..., 1] /= den[1] - 1
    t = t * 8
    return torch.sign(t) * torch.log2(t.abs() + 1.0) / np.log2(8)


def relative_position_index(window):
    """[N, N] int64 (swinv2.py:176-190)."""
    wh, ww = window
    ys, xs = torch.meshgrid(torch.arange(wh), torch.arange(ww), indexing="ij")
    ys, xs = ys.reshape(-1), xs.reshape(-1)
    return (ys[:, None] - ys[None, :] + wh - 1) * (2 * ww - 1) + (xs[:, None] - xs[None, :] + ww - 1)


def shift_attn_mask(H, W, window, shift):
    """[nW, N, N] 0 / -100 region mask (swinv2.py:357-388)."""
    def band(n):
        r = torch.zeros(n, dtype=torch.long)
        r[n - window:n - shift] = 1
        r[n - shift:] = 2
        return r
    reg = 3 * band(H)[:, None] + band(W)[None, :]
    win = reg.reshape(H // window, window, W // window, window).permute(0, 2, 1, 3)
    win = win.reshape(-1, window * window)
    diff = win[:, None, :] != win[:, :, None]
    return torch.zeros(diff.shape).masked_fill(diff, -100.0)


def window_token_index(H, W, window, shift):
    """[nW * N] token index of every (window, position) after roll(-shift) + partition."""
    nwh, nww = H // window, W // window
    k = torch.arange(nwh * nww)
    t = torch.arange(window * window)
    y = ((k // nww)[:, None] * window + (t // window)[None, :] + shift) % H
    x = ((k % nww)[:, None] * window + (t % window)[None, :] + shift) % W
    return (y * W + x).reshape(-1)


# --------------------------------------------------------------------------- modules
class Mlp(nn.Module):
    """fc1 -> GELU -> fc2 (swinv2.py:43-66); runs on bf16 tokens under autocast."""

    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU,
                 drop=0.0):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop = nn.Dropout(drop)

    def forward(self, x):
        return self.drop(ops.linear(self.hidden(x), self.fc2.weight, self.fc2.bias))

    def forward_tokens(self, x, fc2_bias=True):
        """forward() with fc2's bias optional (the caller may fold it into the next kernel);
        fc1 + GELU + fc2 as one autograd node on the fused kernels when dropout is off."""
        b2 = self.fc2.bias if fc2_bias else None
        if (self.drop.p == 0 or not self.training) and isinstance(self.act, nn.GELU) \
                and self.act.approximate == "none":
            return ops.mlp(x, self.fc1.weight, self.fc1.bias, self.fc2.weight, b2)
        return self.drop(ops.linear(self.hidden(x), self.fc2.weight, b2))

    def hidden(self, x):
        """GELU(fc1(x)) with the bias add fused into the activation kernel."""
        if not isinstance(self.act, nn.GELU) or self.act.approximate != "none":
            return self.drop(self.act(ops.linear(x, self.fc1.weight, self.fc1.bias)))
        return self.drop(ops.linear_gelu(x, self.fc1.weight, self.fc1.bias))


class ProjFoldTables(tuple):
    """block_tables()'s fused result (qkv GEMM bias, proj bias, CPB table, logit scale): its proj
    bias holds W_proj v_bias with W_proj detached, so the proj Linear adds that share of
    d proj.weight in its weight-gradient kernel (ops.linear(..., xshift=v_bias))."""


class WindowAttention(nn.Module):
    """W-MSA / SW-MSA with continuous (log-spaced CPB) relative-position bias
    (swinv2.py:105-264).  Parameters and buffers match the reference."""

    def __init__(self, dim, window_size, num_heads, qkv_bias=True, attn_drop=0.0, proj_drop=0.0,
                 pretrained_window_size=[0, 0]):
        super().__init__()
        self.dim = dim
        self.window_size = tuple(window_size)
        self.pretrained_window_size = tuple(pretrained_window_size)
        self.num_heads = num_heads
        if dim % num_heads or dim // num_heads != 32:
            raise NotImplementedError(f"head_dim must be 32 (dim={dim}, heads={num_heads}); "
                                      "every SwinV2 T/S/B/L config uses 32")
        if self.window_size[0] != self.window_size[1]:
            raise NotImplementedError("square windows only")
        self.logit_scale = nn.Parameter(torch.log(10 * torch.ones((num_heads, 1, 1))))
        self.register_buffer("logit_clamp_max", torch.log(torch.tensor(1.0 / 0.01)))
        self._logit_clamp = float(self.logit_clamp_max)  # host copy: no device sync per step
        self.cpb_mlp = nn.Sequential(nn.Linear(2, 512, bias=True), nn.ReLU(inplace=True),
                                     nn.Linear(512, num_heads, bias=False))
        self.register_buffer("relative_coords_table",
                             relative_coords_table(self.window_size, self.pretrained_window_size))
        self.register_buffer("relative_position_index", relative_position_index(self.window_size))
        self.qkv = nn.Linear(dim, dim * 3, bias=False)
        if qkv_bias:
            self.q_bias = nn.Parameter(torch.zeros(dim))
            self.v_bias = nn.Parameter(torch.zeros(dim))
        else:
            self.q_bias = None
            self.v_bias = None
        if attn_drop > 0.0:
            raise NotImplementedError("attention-probability dropout is not fused (reference default 0)")
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)
        self.softmax = nn.Softmax(dim=-1)
        # geometry of the owning block (set by SwinTransformerBlock) for forward(x, mask)
        self.input_resolution = None
        self.shift_size = 0

    # small per-block tables (f32, one fused launch: ops.cpb_table / csrc/cpb.hip)
    def cpb_tables(self):
        """(16*sigmoid(cpb_mlp(relative_coords_table)) as [nH, (2w-1)^2] f32,
        exp(clamp(logit_scale, max=ln 100)) as [nH] f32) (swinv2.py:230, 233-246)."""
        l1, l2 = self.cpb_mlp[0], self.cpb_mlp[2]
        if (isinstance(self.cpb_mlp[1], nn.ReLU) and l1.bias is not None and l2.bias is None
                and l1.out_features == 512 and self.num_heads <= 32):
            return ops.cpb_table(self.relative_coords_table.reshape(-1, 2), l1.weight, l1.bias,
                                 l2.weight, self.logit_scale, self._logit_clamp)
        with torch.autocast(device_type=self.logit_scale.device.type, enabled=False):
            t = self.cpb_mlp(self.relative_coords_table.reshape(-1, 2).float())
            return (16 * torch.sigmoid(t)).t().contiguous(), self.scales()

    def bias_table(self):
        """16*sigmoid(cpb_mlp(relative_coords_table)) as [nH, (2w-1)^2] f32."""
        return self.cpb_tables()[0]

    def scales(self):
        """exp(clamp(logit_scale, max=ln 100)) as [nH] f32 (swinv2.py:230)."""
        return torch.clamp(self.logit_scale, max=self.logit_clamp_max).exp().reshape(-1).float()

    def qkv_gemm_bias(self):
        """Bias of the qkv GEMM: (q_bias, 0, 0), detached.  The reference's bias is
        (q_bias, 0, v_bias) (swinv2.py:218-219); here q_bias's gradient comes out of the W-MSA
        backward kernel (column sums of dq) and v_bias moves into proj_bias()."""
        if self.q_bias is None:
            return None
        z = torch.zeros_like(self.q_bias, requires_grad=False)
        return torch.cat((self.q_bias.detach(), z, z))

    def proj_bias(self):
        """proj.bias + proj.weight @ v_bias: softmax rows sum to 1, so P (V + v_bias) =
        P V + v_bias and v_bias passes through proj as this constant (f32, exact)."""
        if self.v_bias is None:
            return self.proj.bias
        with torch.autocast(device_type=self.v_bias.device.type, enabled=False):
            return self.proj.bias + F.linear(self.v_bias.float(), self.proj.weight.float())

    def gemm_biases(self):
        """(qkv GEMM bias, proj bias) = (qkv_gemm_bias(), proj_bias()), on the GPU as one
        fused launch (ops.attn_biases)."""
        if self.v_bias is not None and self.v_bias.is_cuda:
            return ops.attn_biases(self.q_bias, self.v_bias, self.proj.bias, self.proj.weight)
        return self.qkv_gemm_bias(), self.proj_bias()

    def block_tables(self):
        """(qkv GEMM bias, proj bias, CPB table, logit scale) = gemm_biases() + cpb_tables(),
        on the GPU as one fused launch (ops.block_tables) when both fused forms apply.  The
        fused form returns a `ProjFoldTables`: its proj bias took W_proj detached, so the proj
        Linear that consumes it must add the W_proj v_bias share of the weight gradient itself
        (forward_tokens keys that on the returned object, never on state left behind)."""
        l1, l2 = self.cpb_mlp[0], self.cpb_mlp[2]
        if (self.v_bias is not None and self.v_bias.is_cuda and OPTIONS.block_tables
                and isinstance(self.cpb_mlp[1], nn.ReLU) and l1.bias is not None and l2.bias is None
                and l1.out_features == 512 and self.num_heads <= 32):
            # W_proj enters the folded bias detached: forward_tokens' proj Linear takes the
            # W_proj v_bias share of its weight gradient (xshift = v_bias, one fused kernel)
            return ProjFoldTables(ops.block_tables(
                self.v_bias, self.proj.bias, self.proj.weight.detach(),
                self.relative_coords_table.reshape(-1, 2), l1.weight, l1.bias, l2.weight,
                self.logit_scale, self.q_bias, self._logit_clamp))
        return self.gemm_biases() + self.cpb_tables()

    def forward_tokens(self, x, H, W, shift, proj_bias=True, biases=None, core_only=False):
        """x: bf16 [B, H*W, C] un-partitioned tokens -> [B, H*W, C] after proj (without
        proj's bias when proj_bias=False: the caller folds the proj bias into the next
        kernel).  biases: block_tables() (or gemm_biases()) when the caller already has them.
        core_only: return (o, xshift) -- the attention core's output (proj's input) and the proj
        weight gradient's xshift -- for a caller that runs proj fused with its post-norm."""
        if biases is None:
            biases = self.block_tables()
        qkv_b, proj_b = biases[:2]
        table, scale = biases[2:] if len(biases) == 4 else self.cpb_tables()
        if OPTIONS.qk_epilogue and self.window_size[0] <= 8:
            # q / k normalisation (swinv2.py:229) in the qkv GEMM's epilogue
            qkv, rn = ops.linear_qkv(x, self.qkv.weight, qkv_b, scale)
        else:
            qkv, rn = ops.linear(x, self.qkv.weight, qkv_b), None
        o = ops.window_attention_core(qkv, table, scale, H, W, self.num_heads,
                                      self.window_size[0], shift, q_bias=self.q_bias, rn=rn)
        # the v_bias share of d proj.weight: from this Linear's weight-gradient kernel exactly when
        # the proj bias came from the fused tables (W_proj detached there); gemm_biases() and the
        # unfused tables route it through autograd already
        xshift = self.v_bias if isinstance(biases, ProjFoldTables) else None
        if core_only:
            return o, xshift
        return self.proj_drop(ops.linear(o, self.proj.weight, proj_b if proj_bias else None, xshift=xshift))

    def forward(self, x, mask=None):
        """Reference API (swinv2.py:204): x = windows [nW*B, N, C]."""
        bw, n, c = x.shape
        w = self.window_size[0]
        if mask is None:
            return self.forward_tokens(x, w, w, 0)
        if self.input_resolution is None:
            raise ValueError("a mask needs the owning block's geometry (input_resolution)")
        H, W = self.input_resolution
        nw = mask.shape[0]
        idx = window_token_index(H, W, w, self.shift_size).to(x.device)
        if nw != (H // w) * (W // w) or bw % nw:
            raise ValueError("mask does not match the block geometry")
        b = bw // nw
        tok = torch.empty((b, H * W, c), device=x.device, dtype=x.dtype)
        tok[:, idx] = x.reshape(b, nw * n, c)
        out = self.forward_tokens(tok, H, W, self.shift_size)
        return out[:, idx].reshape(bw, n, c)

    def extra_repr(self):
        return (f"dim={self.dim}, window_size={self.window_size}, "
                f"pretrained_window_size={self.pretrained_window_size}, num_heads={self.num_heads}")

    def flops(self, N):
        return N * self.dim * 3 * self.dim + 2 * self.num_heads * N * (self.dim // self.num_heads) * N \
            + N * self.dim * self.dim


class SwinTransformerBlock(nn.Module):
    """Res-post-norm Swin block (swinv2.py:286-456)."""

    def __init__(self, dim, input_resolution, num_heads, window_size=7, shift_size=0, mlp_ratio=4.0,
                 qkv_bias=True, drop=0.0, attn_drop=0.0, drop_path=0.0, act_layer=nn.GELU,
                 norm_layer=nn.LayerNorm, pretrained_window_size=0):
        super().__init__()
        self.dim = dim
        self.input_resolution = tuple(input_resolution)
        self.num_heads = num_heads
        self.window_size = window_size
        self.shift_size = shift_size
        self.mlp_ratio = mlp_ratio
        if min(self.input_resolution) <= self.window_size:  # swinv2.py:328-331
            self.shift_size = 0
            self.window_size = min(self.input_resolution)
        assert 0 <= self.shift_size < self.window_size, "shift_size must in 0-window_size"
        self.norm1 = norm_layer(dim)
        self.attn = WindowAttention(dim, window_size=to_2tuple(self.window_size), num_heads=num_heads,
                                    qkv_bias=qkv_bias, attn_drop=attn_drop, proj_drop=drop,
                                    pretrained_window_size=to_2tuple(pretrained_window_size))
        self.attn.input_resolution = self.input_resolution
        self.attn.shift_size = self.shift_size
        self.drop_path_prob = float(drop_path)
        self.drop_path = nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = Mlp(in_features=dim, hidden_features=int(dim * mlp_ratio), act_layer=act_layer,
                       drop=drop)
        for n in (self.norm1, self.norm2):
            if not isinstance(n, nn.LayerNorm):
                raise NotImplementedError("the fused post-norm kernel implements nn.LayerNorm")
        H, W = self.input_resolution
        self.register_buffer("attn_mask", shift_attn_mask(H, W, self.window_size, self.shift_size)
                             if self.shift_size > 0 else None)

    def forward_stream(self, s: ResidualStream) -> ResidualStream:
        H, W = self.input_resolution
        B, L, C = s.f32.shape
        assert L == H * W, "input feature has wrong size"
        fold = self.attn.proj_drop.p == 0 or not self.training  # proj bias -> LN kernel
        biases = self.attn.block_tables()
        planned = getattr(self, "_dp", None) if self.training else None  # from _plan_drop_path
        if planned is not None and planned[0].shape[0] != B:
            planned = None
        dev = s.f32.device
        dp = planned[0] if planned else _drop_path_scale(self.drop_path_prob, self.training, B, dev)
        if fold and s.f32.is_cuda and ops.linear_ln_supported(B * L, C, C):
            # stage 0: proj + norm1 (+ DropPath + residual) as one kernel (hvk_linear_ln_fwd)
            o, xshift = self.attn.forward_tokens(s.bf16, H, W, self.shift_size, biases=biases, core_only=True)
            x, xb = ops.linear_ln(o, self.attn.proj.weight, s.f32, self.norm1.weight, self.norm1.bias, dp, L,
                                  self.norm1.eps, abias=biases[1], xshift=xshift)
        else:
            a = self.attn.forward_tokens(s.bf16, H, W, self.shift_size, proj_bias=not fold, biases=biases)
            x, xb = ops.layer_norm_residual(a, s.f32, self.norm1.weight, self.norm1.bias, dp, L,
                                            self.norm1.eps, abias=biases[1] if fold else None)
        fold = self.mlp.drop.p == 0 or not self.training  # fc2 bias -> LN kernel
        dp = planned[1] if planned else _drop_path_scale(self.drop_path_prob, self.training, B, dev)
        m = self.mlp
        if (fold and x.is_cuda and isinstance(m.act, nn.GELU) and m.act.approximate == "none"
                and m.fc1.bias is not None
                and ops.mlp_ln_supported(B * L, C, m.fc1.out_features, m.fc2.out_features)):
            # stage 0: fc1 + GELU + fc2 + norm2 (+ DropPath + residual) as one kernel (hvk_mlp_ln_fwd)
            return ResidualStream(*ops.mlp_ln(xb, m.fc1.weight, m.fc1.bias, m.fc2.weight, x, self.norm2.weight,
                                              self.norm2.bias, dp, L, self.norm2.eps, abias=m.fc2.bias))
        h = m.forward_tokens(xb, fc2_bias=not fold)
        x, xb = ops.layer_norm_residual(h, x, self.norm2.weight, self.norm2.bias, dp, L,
                                        self.norm2.eps, abias=m.fc2.bias if fold else None)
        return ResidualStream(x, xb)

    def forward(self, x):
        return self.forward_stream(_as_stream(x)).f32

    def extra_repr(self):
        return (f"dim={self.dim}, input_resolution={self.input_resolution}, num_heads={self.num_heads}, "
                f"window_size={self.window_size}, shift_size={self.shift_size}, mlp_ratio={self.mlp_ratio}")

    def flops(self):
        H, W = self.input_resolution
        nW = H * W / self.window_size / self.window_size
        return (2 * self.dim * H * W + nW * self.attn.flops(self.window_size * self.window_size)
                + 2 * H * W * self.dim * self.dim * self.mlp_ratio)


class PatchMerging(nn.Module):
    """2x2 gather -> Linear(4C, 2C, no bias) -> LayerNorm(2C) (swinv2.py:459-505)."""

    def __init__(self, input_resolution, dim, norm_layer=nn.LayerNorm):
        super().__init__()
        self.input_resolution = tuple(input_resolution)
        self.dim = dim
        self.reduction = nn.Linear(4 * dim, 2 * dim, bias=False)
        self.norm = norm_layer(2 * dim)

    def forward_stream(self, s: ResidualStream) -> ResidualStream:
        H, W = self.input_resolution
        B, L, C = s.bf16.shape
        assert L == H * W, "input feature has wrong size"
        assert H % 2 == 0 and W % 2 == 0, f"x size ({H}*{W}) are not even."
        if s.bf16.is_cuda and ops.merge_linear_supported(B, H, W, C, 2 * C):
            # the gather folded into the reduction GEMM both ways (no [T/4, 4C] tensor)
            if ops.merge_linear_ln_supported(B, H, W, C, 2 * C):
                x, xb = ops.merge_linear_ln(s.bf16, self.reduction.weight, self.norm.weight, self.norm.bias,
                                            self.norm.eps, H, W)
                return ResidualStream(x, xb)
            y = ops.merge_linear(s.bf16, self.reduction.weight, H, W)
            x, xb = ops.layer_norm_residual(y, None, self.norm.weight, self.norm.bias, None, 1, self.norm.eps)
            return ResidualStream(x, xb)
        xm = ops.patch_merge_gather(s.bf16, H, W)
        if s.bf16.is_cuda and ops.linear_ln_supported(B * L // 4, 4 * C, 2 * C):
            # 2C = 192 (stage 0 -> 1): the reduction GEMM with its norm in the epilogue
            x, xb = ops.linear_ln(xm, self.reduction.weight, None, self.norm.weight, self.norm.bias, None, 1,
                                  self.norm.eps)
            return ResidualStream(x, xb)
        y = ops.linear(xm, self.reduction.weight)
        x, xb = ops.layer_norm_residual(y, None, self.norm.weight, self.norm.bias, None, 1,
                                        self.norm.eps)
        return ResidualStream(x, xb)

    def forward(self, x):
        return self.forward_stream(_as_stream(x)).f32

    def extra_repr(self):
        return f"input_resolution={self.input_resolution}, dim={self.dim}"

    def flops(self):
        H, W = self.input_resolution
        return (H // 2) * (W // 2) * 4 * self.dim * 2 * self.dim + H * W * self.dim // 2


class BasicLayer(nn.Module):
    """One stage: `depth` blocks (even W-MSA, odd SW-MSA) + optional merge (swinv2.py:508-608)."""

    def __init__(self, dim, input_resolution, depth, num_heads, window_size, mlp_ratio=4.0,
                 qkv_bias=True, drop=0.0, attn_drop=0.0, drop_path=0.0, norm_layer=nn.LayerNorm,
                 downsample=None, use_checkpoint=False, pretrained_window_size=0):
        super().__init__()
        self.dim = dim
        self.input_resolution = tuple(input_resolution)
        self.depth = depth
        self.use_checkpoint = use_checkpoint
        self.blocks = nn.ModuleList([
            SwinTransformerBlock(dim=dim, input_resolution=input_resolution, num_heads=num_heads,
                                 window_size=window_size,
                                 shift_size=0 if (i % 2 == 0) else window_size // 2,
                                 mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, drop=drop,
                                 attn_drop=attn_drop,
                                 drop_path=drop_path[i] if isinstance(drop_path, list) else drop_path,
                                 norm_layer=norm_layer, pretrained_window_size=pretrained_window_size)
            for i in range(depth)])
        self.downsample = (downsample(input_resolution, dim=dim, norm_layer=norm_layer)
                           if downsample is not None else None)

    def forward_stream(self, s: ResidualStream) -> ResidualStream:
        for blk in self.blocks:
            if self.use_checkpoint and torch.is_grad_enabled():
                s = ResidualStream(*checkpoint.checkpoint(
                    lambda a, b, m=blk: tuple(m.forward_stream(ResidualStream(a, b))),
                    s.f32, s.bf16, use_reentrant=False))
            else:
                s = blk.forward_stream(s)
        if self.downsample is not None:
            s = self.downsample.forward_stream(s)
        return s

    def forward(self, x):
        return self.forward_stream(_as_stream(x)).f32

    def extra_repr(self):
        return f"dim={self.dim}, input_resolution={self.input_resolution}, depth={self.depth}"

    def flops(self):
        f = sum(b.flops() for b in self.blocks)
        return f + (self.downsample.flops() if self.downsample is not None else 0)

    def _init_respostnorm(self):
        for blk in self.blocks:
            nn.init.constant_(blk.norm1.bias, 0)
            nn.init.constant_(blk.norm1.weight, 0)
            nn.init.constant_(blk.norm2.bias, 0)
            nn.init.constant_(blk.norm2.weight, 0)


class PatchEmbed(nn.Module):
    """4x4/s4 patch projection as a GEMM on token-major patches + LayerNorm (swinv2.py:611-670)."""

    def __init__(self, img_size=224, patch_size=4, in_chans=3, embed_dim=96, norm_layer=None):
        super().__init__()
        img_size, patch_size = to_2tuple(img_size), to_2tuple(patch_size)
        self.img_size = img_size
        self.patch_size = patch_size
        self.patches_resolution = [img_size[0] // patch_size[0], img_size[1] // patch_size[1]]
        self.num_patches = self.patches_resolution[0] * self.patches_resolution[1]
        self.in_chans = in_chans
        self.embed_dim = embed_dim
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.norm = norm_layer(embed_dim) if norm_layer is not None else None
        self.input_norm = None  # (mean, std) f32 [C]: uint8 input normalised here (data.NormalizationFn)

    def set_input_normalization(self, mean, std):
        """Accept the raw uint8 batch of pil_image_collate and apply the device-side
        NormalizationFn (data.py:130-136) inside the patch gather (hvk_patchify_u8_bf16)."""
        dev = self.proj.weight.device
        self.input_norm = (torch.as_tensor(mean, dtype=torch.float32, device=dev).reshape(-1),
                           torch.as_tensor(std, dtype=torch.float32, device=dev).reshape(-1))

    def forward_stream(self, x) -> ResidualStream:
        B, C, H, W = x.shape
        assert H == self.img_size[0] and W == self.img_size[1], \
            f"Input image size ({H}*{W}) doesn't match model ({self.img_size[0]}*{self.img_size[1]})."
        ph, pw = self.patch_size
        gh, gw = self.patches_resolution
        patches = None
        if x.dtype == torch.uint8:
            if self.input_norm is None:
                raise TypeError("uint8 images need set_input_normalization(mean, std) "
                                "(data.NormalizationFn.fuse_into)")
            mean, std = (t.to(x.device) for t in self.input_norm)
            if torch.is_autocast_enabled() and C == 3 and ph == pw == 4:
                patches = ops.patchify_u8_bf16(x, 4, mean, std)  # normalise + cast + gather: one launch
            else:
                x = ops.normalize_u8(x, mean, std)
        if patches is None:
            if (x.is_cuda and torch.is_autocast_enabled() and x.dtype == torch.float32 and C == 3
                    and ph == pw == 4 and not x.requires_grad):
                patches = ops.patchify_bf16(x, 4)  # cast + patch gather in one launch
            else:
                xb = x.to(torch.bfloat16) if torch.is_autocast_enabled() else x
                patches = xb.reshape(B, C, gh, ph, gw, pw).permute(0, 2, 4, 1, 3, 5).reshape(
                    B, gh * gw, C * ph * pw)
        w = self.proj.weight.reshape(self.embed_dim, -1)
        if self.norm is None:
            return _as_stream(ops.linear(patches, w, self.proj.bias))
        if (isinstance(self.norm, nn.LayerNorm) and patches.is_cuda
                and ops.linear_ln_supported(patches.numel() // w.shape[1], w.shape[1], w.shape[0])):
            # the embedding GEMM with its LayerNorm in the epilogue (hvk_linear_ln_fwd, plain norm)
            return ResidualStream(*ops.linear_ln(patches, w, None, self.norm.weight, self.norm.bias, None, 1,
                                                 self.norm.eps, abias=self.proj.bias))
        y = ops.linear(patches, w)
        x32, x16 = ops.layer_norm_residual(y, None, self.norm.weight, self.norm.bias, None, 1,
                                           self.norm.eps, abias=self.proj.bias)
        return ResidualStream(x32, x16)

    def forward(self, x):
        return self.forward_stream(x).f32

    def flops(self):
        Ho, Wo = self.patches_resolution
        f = Ho * Wo * self.embed_dim * self.in_chans * self.patch_size[0] * self.patch_size[1]
        return f + (Ho * Wo * self.embed_dim if self.norm is not None else 0)


def _lib_ln_pool_ok(C):
    """The fused final-norm + pool kernel is built for C (options.norm_pool False: the torch
    form)."""
    from . import _lib
    return OPTIONS.norm_pool and bool(_lib.load().hvk_ln_pool_supported(C))


class SwinTransformerV2(nn.Module):
    """SwinV2 backbone + flat or multitask head (swinv2.py:673-867)."""

    def __init__(self, img_size=224, patch_size=4, in_chans=3, num_classes=1000, embed_dim=96,
                 depths=[2, 2, 6, 2], num_heads=[3, 6, 12, 24], window_size=7, mlp_ratio=4.0,
                 qkv_bias=True, drop_rate=0.0, attn_drop_rate=0.0, drop_path_rate=0.1,
                 norm_layer=nn.LayerNorm, ape=False, patch_norm=True, use_checkpoint=False,
                 pretrained_window_sizes=[0, 0, 0, 0], **kwargs):
        super().__init__()
        self.num_classes = num_classes
        self.num_layers = len(depths)
        self.embed_dim = embed_dim
        self.ape = ape
        self.patch_norm = patch_norm
        self.num_features = int(embed_dim * 2 ** (self.num_layers - 1))
        self.mlp_ratio = mlp_ratio
        self.patch_embed = PatchEmbed(img_size=img_size, patch_size=patch_size, in_chans=in_chans,
                                      embed_dim=embed_dim,
                                      norm_layer=norm_layer if self.patch_norm else None)
        num_patches = self.patch_embed.num_patches
        self.patches_resolution = self.patch_embed.patches_resolution
        if self.ape:
            self.absolute_pos_embed = nn.Parameter(torch.zeros(1, num_patches, embed_dim))
            nn.init.trunc_normal_(self.absolute_pos_embed, std=0.02)
        self.pos_drop = nn.Dropout(p=drop_rate)
        dpr = [x.item() for x in torch.linspace(0, drop_path_rate, sum(depths))]
        self.layers = nn.ModuleList()
        pr = self.patches_resolution
        for i in range(self.num_layers):
            self.layers.append(BasicLayer(
                dim=int(embed_dim * 2 ** i),
                input_resolution=(pr[0] // (2 ** i), pr[1] // (2 ** i)),
                depth=depths[i], num_heads=num_heads[i], window_size=window_size,
                mlp_ratio=self.mlp_ratio, qkv_bias=qkv_bias, drop=drop_rate,
                attn_drop=attn_drop_rate, drop_path=dpr[sum(depths[:i]):sum(depths[:i + 1])],
                norm_layer=norm_layer,
                downsample=PatchMerging if (i < self.num_layers - 1) else None,
                use_checkpoint=use_checkpoint, pretrained_window_size=pretrained_window_sizes[i]))
        self.norm = norm_layer(self.num_features)
        self.avgpool = nn.AdaptiveAvgPool1d(1)
        if isinstance(num_classes, int):
            self.head = nn.Linear(self.num_features, num_classes) if num_classes > 0 else nn.Identity()
            self.hierarchical = False
        else:
            self.num_classes = tuple(num_classes)
            self.head = MultitaskHead(self.num_features, num_classes)
            self.hierarchical = True
        self.apply(self._init_weights)
        for bly in self.layers:
            bly._init_respostnorm()

    def _init_weights(self, m):
        if isinstance(m, nn.Linear):
            nn.init.trunc_normal_(m.weight, std=0.02)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)

    @torch.jit.ignore
    def no_weight_decay(self):
        return {"absolute_pos_embed"}

    @torch.jit.ignore
    def no_weight_decay_keywords(self):
        return {"cpb_mlp", "logit_scale", "relative_position_bias_table"}

    def _plan_drop_path(self, batch, device):
        """Draw every block's two DropPath masks for this forward in one shot ([2n, B]: one
        rand + compare + scale instead of two bernoulli/div launches per residual branch).
        Blocks reuse their pair on an activation-checkpoint recompute."""
        blocks = [blk for layer in self.layers for blk in layer.blocks]
        probs = [blk.drop_path_prob for blk in blocks]
        if not self.training or max(probs, default=0.0) <= 0.0:
            for blk in blocks:
                blk._dp = None
            return
        key = (device, len(blocks))
        if getattr(self, "_dp_keep", None) is None or self._dp_keep[0] != key:
            keep = torch.tensor([1.0 - p for p in probs for _ in (0, 1)], dtype=torch.float32,
                                device=device)
            self._dp_keep = (key, keep)
        keep = self._dp_keep[1][:, None]
        scales = (torch.rand((2 * len(blocks), batch), device=device) < keep).float().div_(keep)
        for i, blk in enumerate(blocks):
            blk._dp = None if probs[i] <= 0.0 else (scales[2 * i], scales[2 * i + 1])

    def _gemm_weights(self):
        """The f32 master weights every GEMM of a forward casts to bf16 (patch embed, qkv,
        proj, fc1, fc2, reductions, a single Linear head), refreshed together by
        ops.prepare_weights."""
        ws = [self.patch_embed.proj.weight.reshape(self.patch_embed.embed_dim, -1)]
        for m in self.modules():
            if isinstance(m, WindowAttention):
                ws += [m.qkv.weight, m.proj.weight]
            elif isinstance(m, Mlp):
                ws += [m.fc1.weight, m.fc2.weight]
            elif isinstance(m, PatchMerging):
                ws.append(m.reduction.weight)
        if isinstance(self.head, nn.Linear):
            ws.append(self.head.weight)
        return [w for w in ws if w.dtype == torch.float32 and w.is_contiguous()]

    def forward_features(self, x, output_activations=False):
        if x.is_cuda:  # one launch for all bf16 weight copies of this step
            ops.prepare_weights(self._gemm_weights())
        self._plan_drop_path(x.shape[0], x.device)
        s = self.patch_embed.forward_stream(x)
        if self.ape:
            s = _as_stream(s.f32 + self.absolute_pos_embed)
        s = ResidualStream(self.pos_drop(s.f32), s.bf16) if self.pos_drop.p > 0 and self.training else s
        acts = [] if output_activations else None
        for layer in self.layers:
            s = layer.forward_stream(s)
            if output_activations:
                acts.append(s.f32)
        if (s.f32.is_cuda and isinstance(self.norm, nn.LayerNorm) and self.norm.elementwise_affine
                and _lib_ln_pool_ok(self.num_features)):
            y = ops.norm_pool(s.f32, self.norm.weight, self.norm.bias, self.norm.eps)  # one kernel
        else:
            if s.f32.is_cuda:
                ops.library_fallback("norm_pool", f"C={self.num_features}")
            with torch.autocast(device_type=x.device.type, enabled=False):
                y = F.layer_norm(s.f32, (self.num_features,), self.norm.weight, self.norm.bias,
                                 self.norm.eps)
            y = y.mean(dim=1)  # avgpool over tokens (swinv2.py:834-835)
        return (y, acts) if output_activations else y

    def _head(self, x):
        """The classifier: a single Linear runs as ops.linear under autocast (the step's
        prepared bf16 weight, f32 dW straight from the GEMM, no per-call casts)."""
        if isinstance(self.head, nn.Linear) and x.is_cuda and torch.is_autocast_enabled():
            if OPTIONS.head_gemm and ops.head_supported(x, [self.head.weight]):
                return ops.head_linear(x, [self.head.weight], [self.head.bias])[0]
            return ops.linear(x, self.head.weight, self.head.bias)
        return self.head(x)

    def forward_head(self, x, pre_logits=False):
        return x if pre_logits else self._head(x)

    def forward(self, x):
        return self._head(self.forward_features(x))

    def flops(self):
        f = self.patch_embed.flops() + sum(layer.flops() for layer in self.layers)
        f += self.num_features * self.patches_resolution[0] * self.patches_resolution[1] // (2 ** self.num_layers)
        if isinstance(self.num_classes, int):
            f += self.num_features * self.num_classes
        else:
            f += sum(self.num_features * n for n in self.num_classes)
        return f


@dataclasses.dataclass(frozen=True)
class Checkpoint:
    """`swin://path` checkpoint URI (swinv2.py:870-895); loads with weights_only=True."""
    source: str
    path: str

    @classmethod
    def parse(cls, uri):
        match = re.match(r"^swin://([\w./-]+)$", uri)
        if not match:
            raise ValueError(f"uri '{uri}' doesn't match the pattern!")
        return cls("swin", match.group(1))

    def load_model_dict(self, cache):
        return self.filter(torch.load(self.path, map_location="cpu", weights_only=True)["model"])

    @staticmethod
    def filter(model_dict):
        ignore = ("relative_position_index", "relative_coords_table", "logit_clamp_max")
        return {k: v for k, v in model_dict.items() if not any(n in k for n in ignore)}
