"""Debug: W-MSA forward vs oracle for one geometry, printing where the mismatches are."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from oracle import swinv2_ref, index_ref  # checker only
import hvamd.ops as ops

B, H, W, nh, win, shift = [int(x) for x in sys.argv[1:7]]
rng = np.random.default_rng(1)
C = 32 * nh
qkv = torch.from_numpy(rng.standard_normal((B, H * W, 3 * C)).astype(np.float32)).bfloat16().float()
tab = torch.from_numpy((16 / (1 + np.exp(-rng.standard_normal((nh, (2 * win - 1) ** 2))))).astype(np.float32))
scale = torch.from_numpy(np.exp(np.minimum(np.log(10) + 0.5 * rng.standard_normal(nh), np.log(100))).astype(np.float32))
ref = swinv2_ref.wmsa_core_ref(qkv, tab, scale, H, W, nh, win, shift)
for rep in range(3):
    out = ops.window_attention_core(qkv.cuda().bfloat16(), tab.cuda(), scale.cuda(), H, W, nh, win, shift).float().cpu()
    err = (out - ref).abs().reshape(B, H, W, nh, 32).amax(-1)
    bad = (err > 0.05).nonzero().tolist()
    print("rep", rep, "rel", ((out - ref).norm() / ref.norm()).item(), "bad", len(bad), bad[:20])
