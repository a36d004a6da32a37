"""Host-side routing switches of the product path, as ONE explicit object.

Every switch here picks between two implementations of the same op that are pinned to each
other by a test (the alternative form exists for A/B measurements and for those tests).  They
are plain attributes of `OPTIONS`, changed only through `set()` / `override()` -- no module of
the package reads the process environment (HVK_LIB_PATH, the library's location, aside) -- and
bench.py prints `as_dict()` into its JSON line, so a result always names the forms it ran.

The library-side forms (tile widths, the ring W-MSA forward, ...) are libhvk options
(`_lib.set_option`, include/hvk.h); `_lib.options()` reads them back the same way.
"""
import contextlib
import dataclasses


@dataclasses.dataclass
class HostOptions:
    # bf16 copies (+ transposes) of every Linear weight made by one launch per step
    # (ops.prepare_weights); False: a cast per Linear call
    prepare_weights: bool = True
    # windows <= 8: q / k normalised (and q pre-scaled) in the qkv GEMM's epilogue
    # (swinv2.py:229-231); False: raw qkv, the W-MSA kernels normalise
    qk_epilogue: bool = True
    # a block's attention biases + CPB table + logit scale as one launch (ops.block_tables)
    block_tables: bool = True
    # classifier / multitask head on libhvk's head GEMM (ops.head_linear)
    head_gemm: bool = True
    # final LayerNorm + token mean pool as one kernel each way (ops.norm_pool)
    norm_pool: bool = True
    # the stage-0 MLP forward / input-gradient chain as one kernel each (hvk_mlp_fwd / _bwd)
    mlp_fused: bool = True
    # C = 96 (stage 0): the post-norm LayerNorm + residual in the epilogue of the proj / fc2 /
    # patch-embedding GEMM (hvk_linear_ln_fwd, hvk_mlp_ln_fwd) instead of a separate launch
    ln_epilogue: bool = True
    # C = 192 (stage 1): the same on the 128 x 192 tile (proj, fc2, the stage-0 -> 1 PatchMerging);
    # needs ln_epilogue.  First form -0.85 % end to end (its 16 dependent norm passes per tile
    # exposed their shuffle / residual-load latency at the tile kernel's 2 waves per SIMD); with two
    # passes interleaved and DPP row sums +0.2 % (3 interleaved pairs on each of two boxes,
    # profiles/round5/ln_epilogue/ab_tile*.txt)
    ln_epilogue_tile: bool = True
    # PatchMerging's 2x2 gather folded into its reduction GEMM (operand loads), the input
    # gradient scattered by the dgrad GEMM's store, the weight gradient gathering on its DMA:
    # no [T/4, 4C] tensor either way (hvk_merge_*, bit-identical)
    merge_gemm: bool = True
    # parameter-gradient launches (weight gradients, the block-bias backward) on a second HIP
    # stream inside the Trainer's backward (ops.wgrad_stream_scope), joined at its end: they
    # overlap the input-gradient chain instead of serialising behind it (+2.6 %, 3 interleaved
    # runs, profiles/round5/wgrad_stream/ab.txt); the Trainer opens the scope for a single rank
    wgrad_stream: bool = True
    # ... including the LayerNorm backward's parameter column sums (hvk_ln_residual_bwd_split):
    # off, measured -1.5 % against the side stream without them (3 interleaved runs,
    # profiles/round5/wgrad_stream/ab_ln.txt)
    wgrad_stream_ln: bool = False
    # ... including the qkv Linear's weight gradient (its bias gradient comes out of the W-MSA
    # backward, so that Linear has no bias gradient of its own; round 5 left it on the main stream)
    wgrad_stream_qkv: bool = True
    # ... also at world > 1, where the bucket all-reduces then start from the side stream: off
    # until RCCL over xGMI says otherwise (the dp2 gloo rehearsal measured -8 %); bench.py
    # --host-opt wgrad_stream_multi_rank=1 is the 8-GPU A/B, its `comm` block the diagnosis
    wgrad_stream_multi_rank: bool = False
    # operands and workspaces of side-stream launches kept alive until the backward's join
    # (ops.wgrad_hold) instead of freed with record_stream, whose blocks the caching allocator
    # reuses only once the GPU has passed their last use: with the host steps ahead (SwinV2-B 384)
    # every step mapped fresh HBM, 287 GB reserved and 470-650 ms per step
    wgrad_hold: bool = True
    # clip + DecoupledSGDW (+ EMA) for every tensor in one fused launch set (hvk_sgdw_step)
    fused_optim: bool = True
    # windows 12 / 16 / 24: the forward keeps its log2 row constants for the backward
    wmsa_large_lse: bool = True
    # SwinV2-B stage 0-1 widths (K = 128 / 256) on the skinny kernel ahead of the tiled one
    skinny_b: bool = True
    # stage-1 fc1 + GELU on the tiled EPI-1 kernel instead of the skinny one (measured -0.1 %)
    s1_gelu_tile: bool = False
    # keep only fc1's h at stage 0 and recompute GELU(h) where consumed (measured -0.4 %)
    gelu_recompute: bool = False
    # a product-path launch that would leave libhvk for a torch / hipBLASLt op (a shape no
    # hand-written kernel takes) raises instead of being counted (ops.library_fallback); the
    # bench-routing parity tests run with it on
    strict_native: bool = False


OPTIONS = HostOptions()
_FIELDS = {f.name: f.type for f in dataclasses.fields(HostOptions)}


def set(**kw):  # noqa: A001 -- options.set(name=value)
    """Set host options by name; returns the previous values (a dict).  Unknown names raise."""
    prev = {}
    for k, v in kw.items():
        if k not in _FIELDS:
            raise KeyError(f"unknown host option {k!r} (known: {sorted(_FIELDS)})")
        prev[k] = getattr(OPTIONS, k)
        setattr(OPTIONS, k, bool(v) if _FIELDS[k] in (bool, "bool") else v)
    return prev


@contextlib.contextmanager
def override(**kw):
    """with options.override(qk_epilogue=False): ... -- restores the previous values."""
    prev = set(**kw)
    try:
        yield OPTIONS
    finally:
        set(**prev)


def parse(text):
    """'name=value' -> {name: value} with value int / bool ('0', '1', 'true', 'false')."""
    name, _, value = text.partition("=")
    name, value = name.strip(), value.strip().lower()
    if name not in _FIELDS:
        raise KeyError(f"unknown host option {name!r} (known: {sorted(_FIELDS)})")
    v = {"true": 1, "false": 0}.get(value)
    return {name: int(value) if v is None else v}


def as_dict():
    return dataclasses.asdict(OPTIONS)


def non_default():
    """The options that differ from the defaults (what a result line must name)."""
    d = HostOptions()
    return {k: v for k, v in as_dict().items() if getattr(d, k) != v}
