"""autograd Functions over libhvk's C ABI (include/hvk.h).

Every Function here launches only HIP kernels from libhvk.so on PyTorch's
current stream; tensors are plumbing (PyTorch owns the memory).  There is no
eager/CPU fallback: a CPU tensor or a missing library raises.
"""
import contextlib
import ctypes

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import call, ptr, stream
from .options import OPTIONS


TIMER_WMSA, TIMER_GEMM, TIMER_ALL = 0x3, 0xC, 0xF  # kind masks (include/hvk.h)


def kernel_timer_start(max_launches=32768, kinds=TIMER_ALL):
    """Time the next W-MSA and / or GEMM launches inside libhvk (dispatch-packet events,
    include/hvk.h); `kinds` is a bit mask of timer kinds."""
    call("hvk_kernel_timer_kinds", int(kinds))
    call("hvk_kernel_timer_enable", int(max_launches))


def kernel_timer_launches(kind):
    """Durations (ms) of the timed launches of one kind, in launch order (call before
    kernel_timer_stop)."""
    out, i = [], 0
    k, t, w = ctypes.c_int(0), ctypes.c_double(0.0), ctypes.c_double(0.0)
    lib = _lib.load()
    while lib.hvk_kernel_timer_launch(i, ctypes.byref(k), ctypes.byref(t), ctypes.byref(w)) == 0:
        if k.value == kind:
            out.append(t.value)
        i += 1
    return out


def kernel_timer_shapes(kinds=(2, 3)):
    """Every timed GEMM launch since kernel_timer_start (call before kernel_timer_stop), in
    launch order: dicts with the kernel family name, kind, M, N, K, algorithmic bytes and flops
    (2 M N K; 4 M N1 K for the fused MLP kernels, as the library records) and duration (ms)."""
    out, i = [], 0
    k, t, w = ctypes.c_int(0), ctypes.c_double(0.0), ctypes.c_double(0.0)
    name = ctypes.create_string_buffer(64)
    mnk, nb = (ctypes.c_double * 3)(), ctypes.c_double(0.0)
    lib = _lib.load()
    while lib.hvk_kernel_timer_launch(i, ctypes.byref(k), ctypes.byref(t), ctypes.byref(w)) == 0:
        if k.value in kinds:
            call("hvk_kernel_timer_launch_shape", i, name, 64, mnk, ctypes.byref(nb))
            out.append({"kernel": name.value.decode(), "kind": k.value, "M": int(mnk[0]), "N": int(mnk[1]),
                        "K": int(mnk[2]), "bytes": nb.value, "flops": w.value, "ms": t.value})
        i += 1
    return out


def kernel_timer_stop():
    """Stop timing; returns {"wmsa_fwd" | "wmsa_bwd" | "gemm" | "wgrad": (total_ms, launches,
    summed algorithmic work)} (GEMM work = 2 M N K flops per launch)."""
    out = {}
    for kind, name in ((0, "wmsa_fwd"), (1, "wmsa_bwd"), (2, "gemm"), (3, "wgrad")):
        t, n, w = ctypes.c_double(0.0), ctypes.c_int(0), ctypes.c_double(0.0)
        call("hvk_kernel_timer_read_work", kind, ctypes.byref(t), ctypes.byref(n), ctypes.byref(w))
        out[name] = (t.value, n.value, w.value)
    call("hvk_kernel_timer_enable", 0)
    return out


def _bf16(t):
    t = t if t.dtype == torch.bfloat16 else t.to(torch.bfloat16)
    return t.contiguous()


def _f32(t):
    t = t if t.dtype == torch.float32 else t.float()
    return t.contiguous()


# --------------------------------------------------------------------------- bf16 weights
class _WeightCopies:
    """bf16 copies (and transposes) of the f32 master weights, refreshed by ONE kernel per
    step (`prepare_weights`, hvk_cast_weights) instead of a cast and a transpose per Linear
    call.  A copy is served only while its master's version counter is unchanged, i.e. until
    the optimizer updates the weight in place; otherwise the Linear casts on the fly."""

    def __init__(self):
        self.key = None
        self.entries = {}
        self.args = None
        self.keep = []

    def prepare(self, weights):
        key = tuple((w.data_ptr(), tuple(w.shape)) for w in weights)
        if key != self.key:
            for w in weights:
                if w.dtype != torch.float32 or w.dim() != 2 or not w.is_contiguous():
                    raise RuntimeError("prepare_weights: contiguous 2-D f32 weights only")
            self.entries, self.keep = {}, []
            srcs, dsts, dts, rows, cols = [], [], [], [], []
            for w in weights:
                N, K = w.shape
                wb = torch.empty((N, K), device=w.device, dtype=torch.bfloat16)
                wt = torch.empty((K, N), device=w.device, dtype=torch.bfloat16)
                self.keep += [wb, wt]
                self.entries[(w.data_ptr(), (N, K))] = [wb, wt, -1]
                srcs.append(ptr(w).value)
                dsts.append(wb.data_ptr())
                dts.append(wt.data_ptr())
                rows.append(N)
                cols.append(K)
            n = len(weights)
            arr = ctypes.c_void_p * n
            self.arrays = (arr(*srcs), arr(*dsts), arr(*dts), (ctypes.c_int * n)(*rows),
                           (ctypes.c_int * n)(*cols))
            self.args = (n,) + tuple(ctypes.cast(a, ctypes.c_void_p) for a in self.arrays)
            self.key = key
        call("hvk_cast_weights", *self.args, stream())
        for w in weights:
            self.entries[(w.data_ptr(), tuple(w.shape))][2] = w._version

    def get(self, w):
        e = self.entries.get((w.data_ptr(), tuple(w.shape)))
        if e is not None and e[2] == w._version and w.dtype == torch.float32:
            return e[0], e[1]
        return None


_WCOPIES = _WeightCopies()


def prepare_weights(weights):
    """Refresh the bf16 copies (+ transposes) of `weights` (f32 [N, K] masters) in one launch;
    the Linear Functions below then use them for this step."""
    if weights and OPTIONS.prepare_weights:
        _WCOPIES.prepare(weights)


def _bf16_weight(w):
    """(bf16 W, bf16 W^T or None) for a Linear weight: the step's prepared copies when they
    are current, else a cast now (the transpose is then made where needed)."""
    c = _WCOPIES.get(w)
    if c is not None:
        return c
    return w.to(torch.bfloat16), None


def _bf16_t(wb, wt):
    return wt if wt is not None else wb.t().contiguous()


# --------------------------------------------------------------------------- Linear
def _split_k_chunks(rows):
    """Chunk count for the weight-gradient reduction over `rows` tokens: a power of two
    dividing rows, chunks of >= 2048 rows, at most 256 chunks."""
    nc = 1
    while nc < 256 and rows % (2 * nc) == 0 and rows // (2 * nc) >= 2048:
        nc *= 2
    return nc


def _gelu_recompute(M, K, N1, N2):
    """With options.gelu_recompute, MlpFn keeps only h = fc1(x) and recomputes GELU(h) inside
    fc2's forward and weight gradient where both kernels are built (stage 0: K 96, N1 384,
    N2 96).  Bit-identical results; off by default: on MI355X the recompute costs fc2 +80 µs
    and its weight gradient +217 µs against the 233 µs the y write saves."""
    lib = _lib.load()
    return (OPTIONS.gelu_recompute and _linear_native(M, K, N1) and lib.hvk_linear_gelu_in_supported(M, N1, N2)
            and lib.hvk_weight_grad_gelu_x_supported(M, N2, N1))


class _WgradStream:
    """options.wgrad_stream state: the side stream, whether a backward that allows it is running
    (wgrad_stream_scope), whether launches on it are not yet joined, whether this backward's join
    callback is queued."""
    side = None
    active = False
    pending = False
    armed = False
    produced = set()  # storage addresses of gradients written on the side stream (until the join)
    held = []  # tensors the side stream reads / writes that the current stream allocated (until the join)
    uses = {}  # id(parameter) -> forward uses since the last backward join (note_leaf_uses)
    forks = 0  # launches put on the side stream (wgrad_fork_count)


def wgrad_fork_count():
    """Parameter-gradient launches placed on the side stream since the process started."""
    return _WgradStream.forks


def note_leaf_uses(leaves, ctx):
    """Count a forward use of each parameter in `leaves` (called by every Function's forward that
    takes parameters; ctx: its context).  A parameter used twice in one graph (tied weights, a
    module called twice) gets two gradients that autograd adds on the current stream, reading
    side-written data without a wait: _wgrad_fork refuses it.  Forwards that build no graph (under
    no_grad: grad mode is off inside every Function.forward, and needs_input_grad follows
    requires_grad only) count as well, which errs on the safe side: until the next reset
    (Trainer, each microbatch) or scope exit such a parameter stays on the current stream."""
    if not (OPTIONS.wgrad_stream and any(ctx.needs_input_grad)):
        return
    for t in leaves:
        if t is not None and t.requires_grad:
            _WgradStream.uses[id(t)] = _WgradStream.uses.get(id(t), 0) + 1


def _flat(leaves):
    """((a, b), (c,)) -> (a, b, c)."""
    out = []
    for t in leaves:
        out.extend(_flat(t) if isinstance(t, tuple) else (t,))
    return tuple(out)


def reset_leaf_uses():
    """Forget the forward-use counts (the Trainer calls it before each microbatch's forward)."""
    _WgradStream.uses.clear()


@contextlib.contextmanager
def wgrad_stream_scope(enabled=True):
    """Around a backward whose parameters all start with .grad None (the Trainer's, after its
    bucket reset, one microbatch): parameter gradients may then be computed on the side stream
    -- autograd hands a fresh leaf gradient over without reading it, and the stream is joined at
    the end of the backward -- so they overlap the input-gradient chain (options.wgrad_stream).
    Outside a scope, or for a parameter that already holds a gradient (accumulation), the launch
    stays on the current stream."""
    prev = _WgradStream.active
    _WgradStream.active = enabled
    try:
        yield
    finally:
        _WgradStream.active = prev
        join_wgrad()
        _WgradStream.uses.clear()


def _side_safe(t):
    """A parameter whose fresh gradient autograd steals without touching it on the current
    stream: a leaf with no gradient yet, f32 (no cast in validate_outputs), contiguous
    (AccumulateGrad steals instead of cloning), no tensor hooks (register_hook runs on the
    current stream; post-accumulate hooks -- GradientBuckets' -- handle the side stream
    themselves) and exactly one forward use since the last join (no autograd-side sum)."""
    return (t.is_leaf and t.grad is None and t.dtype == torch.float32 and t.is_contiguous()
            and not t._backward_hooks and _WgradStream.uses.get(id(t), 0) == 1)


def _wgrad_fork(leaves):
    """(main, side) when the gradients of `leaves` (the parameters the launch produces gradients
    for) may be computed on the side stream, else None."""
    if not (OPTIONS.wgrad_stream and _WgradStream.active and leaves) or torch.cuda.is_current_stream_capturing():
        return None
    if not all(t is None or _side_safe(t) for t in leaves):
        return None
    if _WgradStream.side is None:
        _WgradStream.side = torch.cuda.Stream()
    main = torch.cuda.current_stream()
    _WgradStream.side.wait_stream(main)
    _WgradStream.forks += 1
    return main, _WgradStream.side


def _wgrad_outputs(*ts):
    """Mark gradients a side-stream launch wrote (wgrad_produced_on_side), by storage address:
    AccumulateGrad stores a detached alias (a new tensor object over the same storage)."""
    for t in ts:
        if t is not None:
            _WgradStream.produced.add(t.untyped_storage().data_ptr())


def wgrad_produced_on_side(t):
    """True for a gradient a side-stream launch wrote (since the last join): a consumer on the
    side stream needs no wait for the current stream to read it."""
    return t is not None and t.untyped_storage().data_ptr() in _WgradStream.produced


def wgrad_hold(*tensors):
    """Keep `tensors` (allocated on the current stream, used by side-stream launches) alive until
    the join: dropped right after the current stream has waited for the side stream, their blocks go
    back to the current stream's pool in stream order.  (record_stream instead lets the allocator
    reuse a block only once the GPU has passed its side-stream use: with the host steps ahead of the
    GPU every such block stays unavailable and each step maps fresh HBM -- SwinV2-B 384 went from
    175 to 470-650 ms per step and 287 GB reserved that way.)"""
    if OPTIONS.wgrad_hold:
        _WgradStream.held.extend(t for t in tensors if t is not None)
        return
    side = _WgradStream.side
    for t in tensors:
        if t is not None:
            t.record_stream(side)


def _wgrad_joined(tensors, outputs=()):
    """After launches on the side stream that read / write `tensors` (operands and workspaces,
    allocated on the main stream) and write `outputs` (the gradients handed back to autograd): keep
    the operands alive until the join (wgrad_hold), protect the outputs' memory with record_stream
    (they are small; holding a reference would stop AccumulateGrad from stealing them -- it would
    clone them on the current stream, racing the side stream), and make sure the main stream waits
    for the side stream before the backward returns (an autograd final callback; outside a
    backward, at once)."""
    wgrad_hold(*tensors)
    side = _WgradStream.side
    for t in outputs:
        if t is not None:
            t.record_stream(side)
    _WgradStream.pending = True
    if not _WgradStream.armed:
        try:
            torch.autograd.Variable._execution_engine.queue_callback(_wgrad_join_callback)
            _WgradStream.armed = True
        except RuntimeError:  # not inside a backward pass
            join_wgrad()


def _wgrad_join_callback():
    _WgradStream.armed = False
    join_wgrad()


def join_wgrad():
    """The current stream waits for every weight-gradient launch on the side stream."""
    if _WgradStream.pending:
        torch.cuda.current_stream().wait_stream(_WgradStream.side)
        _WgradStream.pending = False
    _WgradStream.held.clear()  # after the wait: later current-stream reuse is ordered behind the side stream
    _WgradStream.produced.clear()


def wgrad_side_pending():
    """The side stream while launches on it are not joined yet, else None (GradientBuckets'
    hooks then copy each gradient into its bucket on it)."""
    return _WgradStream.side if _WgradStream.pending else None


_DW_TOK = 32  # tokens per stage of libhvk's weight-gradient kernel (csrc/gemm_tn.hip TOK)


def _dw_native(M, N, K, gelu_x=False):
    """libhvk's weight-gradient kernel takes the shape: directly when 32 | M, else as a main launch
    over the first M - M % 32 tokens plus one over the zero-padded 32-token tail (_dw_launch)."""
    lib = _lib.load()
    ok = lib.hvk_weight_grad_gelu_x_supported if gelu_x else lib.hvk_weight_grad_supported
    return M > 0 and bool(ok(M - M % _DW_TOK if M >= _DW_TOK else _DW_TOK, N, K))


def _dw_launch(g, x, with_db, gelu_x, xs, keep):
    """(dW, db) from hvk_weight_grad / _gelu_x / _shift on the current stream; a ragged M (a
    microbatch whose tokens are not a multiple of the kernel's 32-token stage) runs the aligned
    part and the tail padded with zero rows (a zero g row adds nothing; GELU(0) = 0), summed.
    Every tensor the launches touch is appended to `keep` (held until the join: wgrad_hold)."""
    lib = _lib.load()
    M, N = g.shape
    K = x.shape[1]
    dev = g.device

    def one(gg, xx):
        m = gg.shape[0]
        dw = torch.empty((N, K), device=dev, dtype=torch.float32)
        db = torch.empty(N, device=dev, dtype=torch.float32) if with_db else None
        nb = lib.hvk_weight_grad_workspace(m, N, K)
        ws = torch.empty(nb // 4, device=dev, dtype=torch.float32)
        if gelu_x:
            call("hvk_weight_grad_gelu_x", ptr(gg), ptr(xx), ptr(dw), ptr(db), m, N, K, ptr(ws), nb, stream())
        elif xs is not None:
            call("hvk_weight_grad_shift", ptr(gg), ptr(xx), ptr(xs), ptr(dw), ptr(db), m, N, K, ptr(ws), nb, stream())
        else:
            call("hvk_weight_grad", ptr(gg), ptr(xx), ptr(dw), ptr(db), m, N, K, ptr(ws), nb, stream())
        keep.extend((gg, xx, ws))
        return dw, db

    tail = M % _DW_TOK
    if not tail:
        return one(g, x)
    gt = torch.zeros((_DW_TOK, N), device=dev, dtype=g.dtype)
    xt = torch.zeros((_DW_TOK, K), device=dev, dtype=x.dtype)
    gt[:tail].copy_(g[M - tail:])
    xt[:tail].copy_(x[M - tail:])
    dw, db = one(gt, xt)
    if M > tail:
        dw0, db0 = one(g[:M - tail], x[:M - tail])
        keep.extend((gt, xt, dw, db))  # the tail's partials: read by the adds below
        dw = dw0.add_(dw)
        db = db0.add_(db) if with_db else None
    return dw, db


def weight_grad(g, x, with_db=False, gelu_x=False, xshift=None, leaves=()):
    """weight_grad_sync, on the weight-gradient side stream when `leaves` (the parameters whose
    gradients dW / db are) allow it (wgrad_stream_scope) and libhvk's kernel is built for the
    shape, else on the current stream."""
    M, N = g.shape
    K = x.shape[1]
    fork = _wgrad_fork(leaves) if g.is_cuda and _dw_native(M, N, K, gelu_x) else None
    if fork is None:
        return weight_grad_sync(g, x, with_db, gelu_x, xshift)
    main, side = fork
    xs = _f32(xshift) if xshift is not None else None
    keep = [xs]
    with torch.cuda.stream(side):
        dw, db = _dw_launch(g, x, with_db, gelu_x, xs, keep)
    _wgrad_joined(keep, (dw, db))
    _wgrad_outputs(dw, db)
    return dw, db


def weight_grad_sync(g, x, with_db=False, gelu_x=False, xshift=None):
    """(dW, db) = (g^T x, g.sum(0)) in f32 for g [M, N], x [M, K] bf16 with M = tokens (up to
    ~10^6): libhvk's token-chunked MFMA kernel with the bias gradient fused (hvk_weight_grad,
    one pass over g) for every SwinV2 shape it is built for, any M (_dw_launch); otherwise the
    library GEMM batched over token chunks + a small sum, counted as a library fallback.  db is
    None unless with_db.  gelu_x: x holds the fc1 pre-activation h and the kernel contracts with
    GELU(h) (hvk_weight_grad_gelu_x; callers check support).  xshift (f32 [K]) or None:
    dW = g^T (x + 1 xshift^T) (hvk_weight_grad_shift; the proj Linear's folded v_bias)."""
    M, N = g.shape
    K = x.shape[1]
    if gelu_x or _dw_native(M, N, K):
        return _dw_launch(g, x, with_db, gelu_x, _f32(xshift) if xshift is not None else None, [])
    if xshift is not None:
        dw, db = weight_grad(g, x, True)
        dw.add_(torch.outer(db, _f32(xshift)))
        return dw, (db if with_db else None)
    library_fallback("weight_grad", f"M={M} N={N} K={K}")
    db = g.sum(dim=0, dtype=torch.float32) if with_db else None
    nc = _split_k_chunks(M)
    if nc == 1:
        return torch.mm(g.t(), x, out_dtype=torch.float32), db
    kc = M // nc
    part = torch.bmm(g.view(nc, kc, -1).transpose(1, 2), x.view(nc, kc, -1),
                     out_dtype=torch.float32)
    return part.sum(dim=0), db


LIBRARY_FALLBACKS = {}  # site -> launches that left libhvk for a torch / hipBLASLt op


def library_fallback(site, detail=""):
    """Record a product-path launch that leaves libhvk (a shape no hand-written kernel is built
    for); with options.strict_native it raises instead.  bench.py prints the counts and the
    bench-routing tests assert they stay zero."""
    if OPTIONS.strict_native:
        raise RuntimeError(f"library fallback at {site} {detail} (options.strict_native)")
    LIBRARY_FALLBACKS[site] = LIBRARY_FALLBACKS.get(site, 0) + 1


def library_fallbacks(reset=False):
    """{site: count} of library fallbacks since the last reset."""
    out = dict(LIBRARY_FALLBACKS)
    if reset:
        LIBRARY_FALLBACKS.clear()
    return out


_LIN_OK = {}
_TILE_ANY = {}


def _tile_any(M, K, N):
    """libhvk's tiled GEMM takes the shape at all (hvk_gemm_supported: K % 64, 128 | N or 192 | N,
    any M): the native route for shapes outside the measured speed rules of _tile_ok and the
    skinny kernel's table (small microbatches), instead of the library GEMM."""
    ok = _TILE_ANY.get((K, N))
    if ok is None:
        ok = _TILE_ANY[(K, N)] = bool(_lib.load().hvk_gemm_supported(1, K, N))
    return ok and M > 0


def _linear_native(M, K, N):
    """True when libhvk's skinny MFMA GEMM is built for (K, N) (include/hvk.h)."""
    key = (K, N)
    ok = _LIN_OK.get(key)
    if ok is None:
        ok = bool(_lib.load().hvk_linear_supported(max(M, 1), K, N))
        _LIN_OK[key] = ok
    return ok and M > 0


def _tile_ok(M, K, N):
    """libhvk's tiled MFMA GEMM (hvk_gemm_fwd) where it measured faster than the library GEMM
    (tools/bench_gemm.py): the stage-2 shapes (K <= 1536, fc2 forward and fc1 input gradient
    included), the stage-1 shapes with 192 | N (K >= 192), and every stage-3 shape (and the
    stage-2 PatchMerging) with 192 | N, on 128 x 192 tiles."""
    if K % 64 or M <= 0:
        return False
    if N % 128:  # the 128 x 192 tile: stage-1 qkv / proj / fc2 forward, qkv / fc1 input grads
        return N % 192 == 0 and K >= 192 and M >= 32768
    if M >= 8192 and N % 192 == 0:  # stage 3 and its PatchMerging (128 x 192 tiles)
        return True
    return (M >= 32768 and K <= 1536) or (K == 768 and N == 768)


def _native_nt(M, K, N):
    """True when mm_nt runs one of libhvk's GEMMs for this shape."""
    return _tile_ok(M, K, N) or _linear_native(M, K, N) or _tile_any(M, K, N)


def _dgrad_fallback(g2, wb):
    """Input gradient g2 wb for a shape no libhvk GEMM takes (counted / strict, see
    library_fallback)."""
    library_fallback("dgrad", f"M={g2.shape[0]} N={wb.shape[0]} K={wb.shape[1]}")
    return g2 @ wb


def _gelu_skinny_k():
    """fc1 + GELU widths on the skinny kernel (stage 0 outside the fused MLP; stage 1 unless
    options.s1_gelu_tile routes it to the tiled EPI 1 kernel)."""
    return (96,) if OPTIONS.s1_gelu_tile else (96, 192)


def gelu_fwd(x2, wb, bias):
    """(h, GELU(h)) with h = x2 wb^T + bias as ONE kernel (fc1 of swinv2.py:58-62), or None
    when no fused kernel is built for the shape."""
    M, K = x2.shape
    N = wb.shape[0]
    lib = _lib.load()
    if (K in _gelu_skinny_k() or K in _skinny_first_k()) and lib.hvk_linear_gelu_supported(M, K, N):
        fn = "hvk_linear_gelu_fwd"
    elif _tile_any(M, K, N):
        fn = "hvk_gemm_gelu_fwd"
    else:
        return None
    h = torch.empty((M, N), device=x2.device, dtype=torch.bfloat16)
    y = torch.empty_like(h)
    call(fn, ptr(x2), ptr(wb), ptr(_f32(bias)), ptr(h), ptr(y), M, K, N, stream())
    return h, y


def _skinny_first_k():
    """SwinV2-B's stage 0-1 widths (K = 128 / 256): the skinny kernel before the tiled one."""
    return (128, 256) if OPTIONS.skinny_b else ()


def _skinny_first(M, K, N):
    return K in _skinny_first_k() and _linear_native(M, K, N)


def mm_nt(x2, wb, bias=None):
    """y = x2 wb^T (+ bias): libhvk's MFMA kernels -- skinny weight-stationary for the
    memory-bound stage 0-1 shapes, tiled for stages 2-3 (and any other shape the tile takes:
    small microbatches) -- else the library GEMM, counted as a library fallback.  x2 [M, K]
    bf16, wb [N, K] bf16, bias f32 [N]."""
    M, K = x2.shape
    N = wb.shape[0]
    b = _f32(bias) if bias is not None else None
    if (_tile_ok(M, K, N) and not _skinny_first(M, K, N)) or (not _linear_native(M, K, N) and _tile_any(M, K, N)):
        y = torch.empty((M, N), device=x2.device, dtype=torch.bfloat16)
        call("hvk_gemm_fwd", ptr(x2), ptr(wb), ptr(b) if b is not None else None, ptr(y), M, K, N,
             stream())
        return y
    if _linear_native(M, K, N):
        y = torch.empty((M, N), device=x2.device, dtype=torch.bfloat16)
        call("hvk_linear_fwd", ptr(x2), ptr(wb), ptr(b) if b is not None else None, ptr(y), M, K,
             N, stream())
        return y
    library_fallback("mm_nt", f"M={M} K={K} N={N}")
    return F.linear(x2, wb, bias.to(torch.bfloat16) if bias is not None else None)


class LinearFn(torch.autograd.Function):
    """y = x W^T + b with bf16 operands (f32 master W, b); backward returns f32 dW / db
    directly (no bf16 round trip), dW via the split-token batched GEMM.  Forward and input
    gradient run on libhvk's skinny MFMA GEMM for the memory-bound shapes."""

    @staticmethod
    def forward(ctx, x, weight, bias, xshift=None):
        xb = _bf16(x)
        wb, wt = _bf16_weight(weight)
        N, K = wb.shape
        y = mm_nt(xb.reshape(-1, K), wb, bias).reshape(*xb.shape[:-1], N)
        ctx.save_for_backward(xb, wb)
        ctx.wt = wt
        ctx.has_bias = bias is not None
        ctx.xshift = xshift.detach() if xshift is not None else None
        ctx.leaves = (weight, bias)
        note_leaf_uses(_flat(ctx.leaves), ctx)
        return y

    @staticmethod
    def backward(ctx, gy):
        xb, wb = ctx.saved_tensors
        N, K = wb.shape
        g2 = _bf16(gy).reshape(-1, N)
        gx = None
        if ctx.needs_input_grad[0]:
            gx = (mm_nt(g2, _bf16_t(wb, ctx.wt)) if _native_nt(g2.shape[0], N, K)
                  else _dgrad_fallback(g2, wb)).reshape(xb.shape)
        want_db = ctx.has_bias and ctx.needs_input_grad[2]
        dw, db = None, None
        if ctx.needs_input_grad[1]:
            dw, db = weight_grad(g2, xb.reshape(-1, K), want_db, xshift=getattr(ctx, "xshift", None),
                                 leaves=(ctx.leaves[0], ctx.leaves[1] if want_db else None)
                                 if want_db or not ctx.has_bias or OPTIONS.wgrad_stream_qkv else ())
        elif want_db:
            db = g2.sum(dim=0, dtype=torch.float32)
        return gx, dw, db, None


def linear(x, weight, bias=None, xshift=None):
    """F.linear on libhvk's GEMMs.  xshift (detached, [K]) or None: the weight gradient is taken
    for the input x + xshift (the proj Linear, whose v_bias share of the input was folded into
    its bias by block_tables: swinv2.py:255-262)."""
    return LinearFn.apply(x, weight, bias, xshift)


def qkv_nt(x2, wb, bias, scale):
    """(qkv^, rn) for the qkv Linear of a w <= 8 block: y = x2 wb^T + bias with every q and k
    head slice L2-normalised (the F.normalize of swinv2.py:229), q times scale[h] * log2e (the
    attention's logit scale, `scale` f32 [nH]), and rn [M, 2N/96] = their 1 / max(||x||, eps),
    in the GEMM's epilogue where it is built (hvk_linear_qkv_fwd / hvk_gemm_qkv_fwd), else
    mm_nt + hvk_qk_normalize in place."""
    M, K = x2.shape
    N = wb.shape[0]
    lib = _lib.load()
    y = torch.empty((M, N), device=x2.device, dtype=torch.bfloat16)
    rn = torch.empty((M, 2 * N // 96), device=x2.device, dtype=torch.float32)
    b = ptr(_f32(bias)) if bias is not None else None
    sc = _f32(scale.detach())  # its gradient comes from the attention core (logit = scale cos)
    skinny = _linear_native(M, K, N) and lib.hvk_linear_qkv_supported(M, K, N)
    if N % 96 == 0 and ((_tile_ok(M, K, N) and not _skinny_first(M, K, N)) or (not skinny and _tile_any(M, K, N))):
        call("hvk_gemm_qkv_fwd", ptr(x2), ptr(wb), b, ptr(y), ptr(rn), ptr(sc), M, K, N, stream())
    elif skinny:
        call("hvk_linear_qkv_fwd", ptr(x2), ptr(wb), b, ptr(y), ptr(rn), ptr(sc), M, K, N, stream())
    else:
        y = mm_nt(x2, wb, bias)
        call("hvk_qk_normalize", ptr(y), ptr(rn), ptr(sc), M, N // 3, stream())
    return y, rn


class LinearQkvFn(torch.autograd.Function):
    """The qkv Linear with the q / k normalisation (and logit scale) of the attention that
    consumes it (swinv2.py:220 + 229-231): returns (qkv^, rn), see qkv_nt.  Its only consumer,
    WindowAttentionCore with rn, returns the gradient with respect to the UN-normalised qkv
    (hvk_wmsa_bwd_normed applies the normalisation's backward), so the backward here is
    LinearFn's."""

    @staticmethod
    def forward(ctx, x, weight, bias, scale):
        xb = _bf16(x)
        wb, wt = _bf16_weight(weight)
        N, K = wb.shape
        y, rn = qkv_nt(xb.reshape(-1, K), wb, bias, scale)
        ctx.save_for_backward(xb, wb)
        ctx.wt = wt
        ctx.has_bias = bias is not None
        ctx.leaves = (weight, bias)
        note_leaf_uses(_flat(ctx.leaves), ctx)
        ctx.mark_non_differentiable(rn)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for rn (one fill per block)
        return y.reshape(*xb.shape[:-1], N), rn

    @staticmethod
    def backward(ctx, gy, grn):
        if gy is None:
            return None, None, None, None
        return LinearFn.backward(ctx, gy)  # (gx, dW, db, None for scale)


def linear_qkv(x, weight, bias, scale):
    """The qkv Linear with q, k normalised and q pre-scaled by the attention's logit scale
    (`scale` [nH], detached here: its gradient comes from window_attention_core).

    Gradient contract (non-standard): the returned qkv^ must be consumed ONLY by
    window_attention_core(..., rn=rn), whose backward returns the gradient with respect to the
    UN-normalised qkv -- the one LinearQkvFn.backward expects.  Any other consumer would get
    wrong gradients, so the output is tagged and window_attention_core refuses an rn paired with
    an untagged qkv."""
    y, rn = LinearQkvFn.apply(x, weight, bias, scale)
    y._hvk_qk_normed = True
    return y, rn


# --------------------------------------------------------------------------- classifier head
_HEAD_WS = {}
_HEAD_W = {}  # device -> (key, concatenated bf16 tier weights): rebuilt only when a weight changes


def _head_weight(ws, K, Np, device):
    """The tiers' bf16 weights concatenated (and zero-padded to Np rows) once per optimizer
    update, keyed on the f32 masters' storage and version counters, instead of a fresh
    [Np, K] copy every forward (15 MB for a 10 000-class head)."""
    if len(ws) == 1 and ws[0].shape[0] == Np:
        return _bf16_weight(ws[0])[0]
    key = tuple((w.data_ptr(), w._version, tuple(w.shape)) for w in ws) + (Np, K)
    c = _HEAD_W.get(device)
    if c is not None and c[0] == key:
        return c[1]
    buf = torch.zeros((Np, K), device=device, dtype=torch.bfloat16)
    off = 0
    for w in ws:
        buf[off:off + w.shape[0]].copy_(_bf16_weight(w)[0])
        off += w.shape[0]
    _HEAD_W[device] = (key, buf)
    return buf


class HeadFn(torch.autograd.Function):
    """The classifier head (swinv2.py:786-794) or the multitask tiers (hierarchy.py:19-47) as
    ONE libhvk GEMM over their concatenated classes (hvk_head_fwd / hvk_head_bwd): logits
    [M, N_t] per tier (views of one [M, N_pad] bf16 output, N_pad = sum N_t rounded up to 8 with
    zero weight rows), f32 dW / db straight from the kernels.  x: [M, K] pooled features."""

    @staticmethod
    def forward(ctx, x, n_w, *wb):
        note_leaf_uses(wb, ctx)
        ws, bs = wb[:n_w], wb[n_w:]
        xb = _bf16(x).contiguous()
        M, K = xb.shape
        sizes = [w.shape[0] for w in ws]
        N = sum(sizes)
        Np = (N + 7) // 8 * 8
        wcat = _head_weight(ws, K, Np, xb.device)
        has_b = all(b is not None for b in bs) and len(bs) == n_w
        bcat = None
        if has_b:
            bl = [_f32(b) for b in bs] + ([torch.zeros(Np - N, device=xb.device)] if Np != N else [])
            bcat = bl[0] if len(bl) == 1 else torch.cat(bl)
        y = torch.empty((M, Np), device=xb.device, dtype=torch.bfloat16)
        call("hvk_head_fwd", ptr(xb), ptr(wcat), ptr(bcat) if has_b else None, ptr(y), M, K, Np, stream())
        ctx.save_for_backward(xb, wcat)
        ctx.sizes, ctx.Np, ctx.has_b, ctx.n_w = sizes, Np, has_b, n_w
        ctx.x_dtype = x.dtype
        outs, off = [], 0
        for n in sizes:
            outs.append(y[:, off:off + n])
            off += n
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gys):
        xb, wcat = ctx.saved_tensors
        M, K = xb.shape
        sizes, Np = ctx.sizes, ctx.Np
        parts = [(_bf16(g) if g is not None else torch.zeros((M, n), device=xb.device, dtype=torch.bfloat16))
                 for g, n in zip(gys, sizes)]
        if Np != sum(sizes):
            parts.append(torch.zeros((M, Np - sum(sizes)), device=xb.device, dtype=torch.bfloat16))
        g = parts[0].contiguous() if len(parts) == 1 else torch.cat(parts, dim=1)
        want_x = ctx.needs_input_grad[0]
        want_w = any(ctx.needs_input_grad[2:2 + ctx.n_w])
        want_b = ctx.has_b and any(ctx.needs_input_grad[2 + ctx.n_w:])
        gx = torch.empty((M, K), device=xb.device, dtype=torch.float32) if want_x else None
        dw = torch.empty((Np, K), device=xb.device, dtype=torch.float32) if (want_w or want_b) else None
        db = torch.empty(Np, device=xb.device, dtype=torch.float32) if want_b else None
        nb = _lib.load().hvk_head_bwd_workspace_bytes(M, K, Np) if want_x else 0
        key = (xb.device, nb)
        wsb = _HEAD_WS.get(key)
        if nb and wsb is None:
            wsb = _HEAD_WS[key] = torch.empty(nb // 4, device=xb.device, dtype=torch.float32)
        call("hvk_head_bwd", ptr(g), ptr(xb), ptr(wcat), ptr(gx) if want_x else None, ptr(dw) if dw is not None else None,
             ptr(db) if want_b else None, M, K, Np, ptr(wsb) if nb else None, nb, stream())
        dws, dbs, off = [], [], 0
        for n in sizes:
            dws.append(dw[off:off + n] if want_w else None)
            dbs.append(db[off:off + n] if want_b else None)
            off += n
        if not ctx.has_b:
            dbs = [None] * (len(ctx.needs_input_grad) - 2 - ctx.n_w)
        gx = gx.to(ctx.x_dtype) if want_x and ctx.x_dtype != torch.float32 else gx
        return (gx, None, *dws, *dbs)


def head_supported(x, weights):
    """True when the libhvk head GEMMs take this head: CUDA, 2-D features, K % 8 == 0."""
    if not x.is_cuda or x.dim() != 2:
        return False
    K = x.shape[1]
    N = (sum(w.shape[0] for w in weights) + 7) // 8 * 8
    return bool(_lib.load().hvk_head_supported(x.shape[0], K, N))


def head_linear(x, weights, biases):
    """Logits of every head Linear (weights[t] [N_t, K], biases[t] [N_t] or None) in one GEMM:
    a tuple of bf16 [M, N_t] (views of one buffer)."""
    bs = list(biases) if all(b is not None for b in biases) else []
    return HeadFn.apply(x, len(weights), *weights, *bs)


# --------------------------------------------------------------------------- block biases
class AttnBiasFn(torch.autograd.Function):
    """(qkv GEMM bias (q_bias, 0, 0), proj bias + W_proj v_bias) of a W-MSA block in ONE
    launch (hvk_attn_bias_fwd) and its backward in one more, instead of zeros + cat + a
    GEMV + an add forward and the matching autograd chain backward (swinv2.py:218-220, 262).
    q_bias enters detached: its gradient is the W-MSA backward's column sums of dq."""

    @staticmethod
    def forward(ctx, v_bias, proj_bias, proj_w, q_bias):
        note_leaf_uses((v_bias, proj_bias, proj_w), ctx)
        C = v_bias.numel()
        v, w = _f32(v_bias), _f32(proj_w)
        pb = _f32(proj_bias) if proj_bias is not None else None
        qb = _f32(q_bias.detach()) if q_bias is not None else None
        qkv_bias = torch.empty(3 * C, device=v.device, dtype=torch.float32)
        eff = torch.empty(C, device=v.device, dtype=torch.float32)
        dv = torch.empty(C, device=v.device, dtype=torch.float32)  # zeroed by the launch
        call("hvk_attn_bias_fwd", ptr(qb), ptr(v), ptr(pb), ptr(w), C, ptr(qkv_bias), ptr(eff),
             ptr(dv), stream())
        ctx.save_for_backward(v, w)
        ctx.dv = dv
        ctx.has_pb = proj_bias is not None
        ctx.mark_non_differentiable(qkv_bias)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the qkv bias output
        return qkv_bias, eff

    @staticmethod
    def backward(ctx, g_qkv, g_eff):
        v, w = ctx.saved_tensors
        if g_eff is None:
            return None, None, None, None
        g = _f32(g_eff)
        C = v.numel()
        dpb = torch.empty_like(g) if ctx.has_pb else None
        dv, dw = ctx.dv, torch.empty_like(w)
        ctx.dv = None  # the only reference left is the returned one: AccumulateGrad steals it
        call("hvk_attn_bias_bwd", ptr(g), ptr(v), ptr(w), C, ptr(dpb), ptr(dv), ptr(dw), stream())
        return dv, dpb, dw, None


def attn_biases(q_bias, v_bias, proj_bias, proj_w):
    return AttnBiasFn.apply(v_bias, proj_bias, proj_w, q_bias)


# --------------------------------------------------------------------------- W-MSA
_WMSA_WS = {}


def _wmsa_workspace(device, nbytes):
    """Persistent zero-filled W-MSA backward workspace (the kernels leave it zero again,
    include/hvk.h), one per device and size: no memset per call."""
    key = (device, nbytes)
    ws = _WMSA_WS.get(key)
    if ws is None:
        ws = torch.zeros(nbytes // 4, device=device, dtype=torch.float32)
        _WMSA_WS[key] = ws
    return ws


class WindowAttentionCore(torch.autograd.Function):
    """Shifted-window cosine attention core on un-partitioned tokens.

    qkv [B, H*W, 3C] bf16 (bias (q_bias, 0, 0) already in it) -> out [B, H*W, C] bf16,
    without v_bias (the caller folds proj.weight @ v_bias into proj's bias).  Stands in for
    swinv2.py:399-412 + 221-261 + 420-429 (see include/hvk.h).  `q_bias` is taken only to
    route its gradient: d loss / d q_bias = column sums of dq, produced by the backward
    kernel (the qkv GEMM gets the bias detached, so no separate reduction runs).  For windows
    12 / 16 / 24 the forward also keeps each query's softmax
    row constant (4 B per token and head) and the backward takes it with the output (kept
    anyway as proj's saved input) instead of recomputing the row statistics."""

    @staticmethod
    def forward(ctx, qkv, q_bias, bias_table, scale, H, W, num_heads, window, shift, rn=None):
        note_leaf_uses((q_bias,), ctx)
        B, L, C3 = qkv.shape
        C = C3 // 3
        if L != H * W:
            raise ValueError(f"token count {L} != {H}*{W}")
        qkv = _bf16(qkv)
        bias_table = _f32(bias_table)
        scale = _f32(scale)
        out = torch.empty((B, L, C), device=qkv.device, dtype=torch.bfloat16)
        ctx.geom = (B, H, W, C, num_heads, window, shift)
        ctx.has_q_bias = q_bias is not None
        if rn is not None:  # q^, k^ from linear_qkv
            call("hvk_wmsa_fwd_normed", ptr(qkv), ptr(out), ptr(bias_table), ptr(scale), B, H, W, C,
                 num_heads, window, shift, stream())
            ctx.save_for_backward(qkv, bias_table, scale, rn)
            return out
        # windows 12 / 16 / 24: the forward keeps the row constants and the backward skips its
        # row-statistics pass (options.wmsa_large_lse False: recompute them)
        keep = OPTIONS.wmsa_large_lse and window > 8
        lse = torch.empty((B, L, num_heads), device=qkv.device, dtype=torch.float32) if keep else None
        call("hvk_wmsa_fwd", ptr(qkv), ptr(out), ptr(lse), ptr(bias_table), ptr(scale), B, H, W, C,
             num_heads, window, shift, stream())
        if lse is not None:
            ctx.save_for_backward(qkv, bias_table, scale, out, lse)
        else:
            ctx.save_for_backward(qkv, bias_table, scale)
        return out

    @staticmethod
    def backward(ctx, dout):
        saved = ctx.saved_tensors
        qkv, bias_table, scale = saved[:3]
        B, H, W, C, nh, win, shift = ctx.geom
        if len(saved) == 4:
            return WindowAttentionCore._backward_normed(ctx, dout, qkv, bias_table, scale, saved[3])
        out, lse = saved[3:] if len(saved) == 5 else (None, None)
        dout = _bf16(dout)
        dqkv = torch.empty_like(qkv)
        dtab = torch.empty_like(bias_table)
        dscale = torch.empty_like(scale)
        dqb = (torch.empty(C, device=qkv.device, dtype=torch.float32)
               if ctx.has_q_bias and ctx.needs_input_grad[1] else None)
        ws_bytes = _lib.load().hvk_wmsa_bwd_workspace_bytes(nh, win)
        ws = _wmsa_workspace(qkv.device, ws_bytes)
        call("hvk_wmsa_bwd", ptr(qkv), ptr(dout), ptr(out), ptr(lse), ptr(dqkv),
             ptr(dqb) if dqb is not None else None, ptr(bias_table), ptr(scale), ptr(dtab),
             ptr(dscale), ptr(ws), ws_bytes, B, H, W, C, nh, win, shift, stream())
        return dqkv, dqb, dtab, dscale, None, None, None, None, None, None

    @staticmethod
    def _backward_normed(ctx, dout, qkv, bias_table, scale, rn):
        B, H, W, C, nh, win, shift = ctx.geom
        dout = _bf16(dout)
        dqkv = torch.empty_like(qkv)
        dtab = torch.empty_like(bias_table)
        dscale = torch.empty_like(scale)
        dqb = (torch.empty(C, device=qkv.device, dtype=torch.float32)
               if ctx.has_q_bias and ctx.needs_input_grad[1] else None)
        ws_bytes = _lib.load().hvk_wmsa_bwd_workspace_bytes(nh, win)
        ws = _wmsa_workspace(qkv.device, ws_bytes)
        call("hvk_wmsa_bwd_normed", ptr(qkv), ptr(rn), ptr(dout), ptr(dqkv),
             ptr(dqb) if dqb is not None else None, ptr(bias_table), ptr(scale), ptr(dtab),
             ptr(dscale), ptr(ws), ws_bytes, B, H, W, C, nh, win, shift, stream())
        return dqkv, dqb, dtab, dscale, None, None, None, None, None, None


def window_attention_core(qkv, bias_table, scale, H, W, num_heads, window, shift, q_bias=None, rn=None):
    """rn given: qkv holds (q^, k^, v) from linear_qkv (windows <= 8) and the gradient returned
    for it is the one with respect to the un-normalised qkv."""
    if rn is not None and not getattr(qkv, "_hvk_qk_normed", False):
        raise ValueError("window_attention_core(rn=...) takes the qkv^ returned by linear_qkv itself "
                         "(its backward returns the gradient of the un-normalised qkv)")
    return WindowAttentionCore.apply(qkv, q_bias, bias_table, scale, H, W, num_heads, window,
                                     shift, rn)


# --------------------------------------------------------------------------- CPB table
_CPB_WS = {}


class CpbTable(torch.autograd.Function):
    """(table [nH, RR], scale [nH]) = (16 sigmoid(cpb_mlp(coords)) transposed, exp(clamp(
    logit_scale))) in one launch (hvk_cpb_fwd); backward two launches (hvk_cpb_bwd).
    Replaces swinv2.py:230 and 233-246 (before the rpi gather)."""

    @staticmethod
    def forward(ctx, coords, w1, b1, w2, logit_scale, clamp_max):
        note_leaf_uses((w1, b1, w2, logit_scale), ctx)
        coords, w1, b1, w2 = _f32(coords), _f32(w1), _f32(b1), _f32(w2)
        logit = _f32(logit_scale.reshape(-1))
        nH, hid = w2.shape
        RR = coords.shape[0]
        table = torch.empty((nH, RR), device=w1.device, dtype=torch.float32)
        scale = torch.empty(nH, device=w1.device, dtype=torch.float32)
        call("hvk_cpb_fwd", ptr(coords), ptr(w1), ptr(b1), ptr(w2), ptr(logit), float(clamp_max),
             RR, nH, hid, ptr(table), ptr(scale), stream())
        ctx.save_for_backward(coords, w1, b1, w2, logit, table)
        ctx.clamp_max = float(clamp_max)
        ctx.logit_shape = logit_scale.shape
        return table, scale

    @staticmethod
    def backward(ctx, dtable, dscale):
        coords, w1, b1, w2, logit, table = ctx.saved_tensors
        nH, hid = w2.shape
        RR = coords.shape[0]
        dtable = _f32(dtable) if dtable is not None else torch.zeros_like(table)
        dscale = _f32(dscale) if dscale is not None else torch.zeros_like(logit)
        dw1, db1, dw2 = torch.empty_like(w1), torch.empty_like(b1), torch.empty_like(w2)
        dlogit = torch.empty_like(logit)
        nbytes = _lib.load().hvk_cpb_bwd_workspace_bytes(RR, nH)
        key = (w1.device, nbytes)
        ws = _CPB_WS.get(key)
        if ws is None:
            ws = _CPB_WS[key] = torch.empty(nbytes // 4, device=w1.device, dtype=torch.float32)
        call("hvk_cpb_bwd", ptr(coords), ptr(w1), ptr(b1), ptr(w2), ptr(logit), ctx.clamp_max, RR,
             nH, hid, ptr(table), ptr(dtable), ptr(dscale), ptr(dw1), ptr(db1), ptr(dw2),
             ptr(dlogit), ptr(ws), nbytes, stream())
        return None, dw1, db1, dw2, dlogit.reshape(ctx.logit_shape), None


def cpb_table(coords, w1, b1, w2, logit_scale, clamp_max):
    return CpbTable.apply(coords, w1, b1, w2, logit_scale, clamp_max)


class BlockTables(torch.autograd.Function):
    """AttnBiasFn + CpbTable of one W-MSA block in one launch forward (hvk_block_bias_fwd)
    and two backward (hvk_block_bias_bwd): (qkv GEMM bias, proj bias + W_proj v_bias, CPB
    table [nH, RR], logit scale [nH]); same kernels' bodies, same results."""

    @staticmethod
    def forward(ctx, v_bias, proj_bias, proj_w, coords, w1, b1, w2, logit_scale, q_bias, clamp_max):
        C = v_bias.numel()
        v, pw = _f32(v_bias), _f32(proj_w)
        pb = _f32(proj_bias) if proj_bias is not None else None
        qb = _f32(q_bias.detach()) if q_bias is not None else None
        coords, w1, b1, w2 = _f32(coords), _f32(w1), _f32(b1), _f32(w2)
        logit = _f32(logit_scale.reshape(-1))
        nH, hid = w2.shape
        RR = coords.shape[0]
        dev = v.device
        qkv_bias = torch.empty(3 * C, device=dev, dtype=torch.float32)
        eff = torch.empty(C, device=dev, dtype=torch.float32)
        dv = torch.empty(C, device=dev, dtype=torch.float32)  # zeroed by the launch
        table = torch.empty((nH, RR), device=dev, dtype=torch.float32)
        scale = torch.empty(nH, device=dev, dtype=torch.float32)
        call("hvk_block_bias_fwd", ptr(qb), ptr(v), ptr(pb), ptr(pw), C, ptr(coords), ptr(w1), ptr(b1),
             ptr(w2), ptr(logit), float(clamp_max), RR, nH, hid, ptr(qkv_bias), ptr(eff), ptr(dv),
             ptr(table), ptr(scale), stream())
        ctx.save_for_backward(v, pw, coords, w1, b1, w2, logit, table)
        ctx.dv = dv
        ctx.has_pb = proj_bias is not None
        ctx.clamp_max = float(clamp_max)
        ctx.logit_shape = logit_scale.shape
        ctx.leaves = (v_bias, proj_bias, proj_w, w1, b1, w2, logit_scale)
        note_leaf_uses(_flat(ctx.leaves), ctx)
        ctx.mark_non_differentiable(qkv_bias)
        ctx.set_materialize_grads(False)
        return qkv_bias, eff, table, scale

    @staticmethod
    def backward(ctx, g_qkv, g_eff, dtable, dscale):
        v, pw, coords, w1, b1, w2, logit, table = ctx.saved_tensors
        C = v.numel()
        nH, hid = w2.shape
        RR = coords.shape[0]
        dv, dpw, dpb = None, None, None
        if g_eff is not None:
            g_eff = _f32(g_eff)
            # proj_w passed detached: its v_bias share is added by the proj Linear's weight-gradient
            # kernel (linear(..., xshift=v_bias)), no separate C x C gradient and accumulation here
            dv, dpw = ctx.dv, (torch.empty_like(pw) if ctx.needs_input_grad[2] else None)
            dpb = torch.empty_like(g_eff) if ctx.has_pb else None
        ctx.dv = None  # the returned d v_bias is then its only reference: AccumulateGrad steals it
        dtable = _f32(dtable) if dtable is not None else torch.zeros_like(table)
        dscale = _f32(dscale) if dscale is not None else torch.zeros_like(logit)
        dw1, db1, dw2 = torch.empty_like(w1), torch.empty_like(b1), torch.empty_like(w2)
        dlogit = torch.empty_like(logit)
        nbytes = _lib.load().hvk_cpb_bwd_workspace_bytes(RR, nH)
        key = (w1.device, nbytes)
        ws = _CPB_WS.get(key)
        if ws is None:
            ws = _CPB_WS[key] = torch.empty(nbytes // 4, device=w1.device, dtype=torch.float32)
        # parameter gradients only: on the weight-gradient side stream when enabled
        fork = _wgrad_fork(ctx.leaves)
        with torch.cuda.stream(fork[1]) if fork else contextlib.nullcontext():
            call("hvk_block_bias_bwd", ptr(g_eff), ptr(v), ptr(pw), C, ptr(dpb), ptr(dv), ptr(dpw),
                 ptr(coords), ptr(w1), ptr(b1), ptr(w2), ptr(logit), ctx.clamp_max, RR, nH, hid, ptr(table),
                 ptr(dtable), ptr(dscale), ptr(dw1), ptr(db1), ptr(dw2), ptr(dlogit), ptr(ws), nbytes,
                 stream())
        if fork:
            _wgrad_joined((g_eff, v, pw, coords, w1, b1, w2, logit, table, dtable, dscale),
                          (dpb, dv, dpw, dw1, db1, dw2, dlogit))
            _wgrad_outputs(dv, dpb, dpw, dw1, db1, dw2)
        return (dv, dpb, dpw, None, dw1, db1, dw2, dlogit.reshape(ctx.logit_shape), None, None)


def block_tables(v_bias, proj_bias, proj_w, coords, w1, b1, w2, logit_scale, q_bias, clamp_max):
    return BlockTables.apply(v_bias, proj_bias, proj_w, coords, w1, b1, w2, logit_scale, q_bias,
                             clamp_max)


# --------------------------------------------------------------------------- LayerNorm
class LayerNormResidual(torch.autograd.Function):
    """x = x0 + s[b] * LayerNorm(a + abias); returns (x f32, x bf16 copy).  abias is the
    bias of the Linear that produced `a` (that GEMM runs without it)."""

    @staticmethod
    def forward(ctx, a, abias, x0, gamma, beta, sample_scale, rows_per_sample, eps):
        abias_p, gamma_p, beta_p = abias, gamma, beta
        C = a.shape[-1]
        rows = a.numel() // C
        a = _bf16(a)
        gamma, beta = _f32(gamma), _f32(beta)
        abias = _f32(abias) if abias is not None else None
        x0 = _f32(x0) if x0 is not None else None
        sample_scale = _f32(sample_scale) if sample_scale is not None else None
        x = torch.empty(a.shape, device=a.device, dtype=torch.float32)
        xb = torch.empty(a.shape, device=a.device, dtype=torch.bfloat16)
        mean = torch.empty(rows, device=a.device, dtype=torch.float32)
        rstd = torch.empty(rows, device=a.device, dtype=torch.float32)
        call("hvk_ln_residual_fwd", ptr(a), ptr(abias), ptr(x0), ptr(gamma), ptr(beta),
             ptr(sample_scale), rows, C, rows_per_sample, float(eps), ptr(x), ptr(xb), ptr(mean),
             ptr(rstd), stream())
        ctx.save_for_backward(a, abias, gamma, sample_scale, mean, rstd)
        ctx.ln_leaves = (abias_p, gamma_p, beta_p)
        note_leaf_uses(_flat(ctx.ln_leaves), ctx)
        ctx.has_x0 = x0 is not None
        ctx.rps = rows_per_sample
        # an unused output (e.g. the bf16 copy at a stage end) gets None, not a zero-filled
        # activation-sized gradient: the kernel takes NULL for either
        ctx.set_materialize_grads(False)
        return x, xb

    @staticmethod
    def backward(ctx, gx, gxb):
        a, abias, gamma, sample_scale, mean, rstd = ctx.saved_tensors
        r = _ln_residual_bwd(a, abias, gamma, sample_scale, mean, rstd, ctx.rps, ctx.has_x0, gx, gxb, ctx.ln_leaves)
        if r is None:
            return (None,) * 8
        ga, dabias, gx0, dgamma, dbeta = r
        return ga, dabias, gx0, dgamma, dbeta, None, None, None


def _ln_residual_bwd(a, abias, gamma, sample_scale, mean, rstd, rps, has_x0, gx, gxb, leaves=()):
    """Backward of x = x0 + s (gamma * LN(a + abias) + beta) (hvk_ln_residual_bwd): (ga, dabias,
    gx0, dgamma, dbeta), or None when neither output has a gradient.  `leaves`: the parameters
    (abias, gamma, beta) whose gradients the column sums are; where they allow it
    (wgrad_stream_scope) the sums run on the side stream (hvk_ln_residual_bwd_split)."""
    C = a.shape[-1]
    rows = a.numel() // C
    gx = _f32(gx) if gx is not None else None
    gxb = _bf16(gxb) if gxb is not None else None
    if gx is None and gxb is None:
        return None
    ga = torch.empty_like(a)
    gx0 = torch.empty(a.shape, device=a.device, dtype=torch.float32) if has_x0 else None
    dgamma = torch.empty_like(gamma)
    dbeta = torch.empty_like(gamma)
    dabias = torch.empty_like(gamma) if abias is not None else None
    ws_bytes = _lib.load().hvk_ln_bwd_workspace_bytes(C)
    ws = torch.empty(ws_bytes // 4, device=a.device, dtype=torch.float32)
    fork = _wgrad_fork(leaves) if a.is_cuda and OPTIONS.wgrad_stream_ln else None
    if fork is None:
        call("hvk_ln_residual_bwd", ptr(a), ptr(abias), ptr(gamma), ptr(sample_scale), ptr(mean),
             ptr(rstd), ptr(gx), ptr(gxb), rows, C, rps, ptr(gx0), ptr(ga), ptr(dgamma),
             ptr(dbeta), ptr(dabias), ptr(ws), ws_bytes, stream())
        return ga, dabias, gx0, dgamma, dbeta
    call("hvk_ln_residual_bwd_split", ptr(a), ptr(abias), ptr(gamma), ptr(sample_scale), ptr(mean),
         ptr(rstd), ptr(gx), ptr(gxb), rows, C, rps, ptr(gx0), ptr(ga), ptr(dgamma),
         ptr(dbeta), ptr(dabias), ptr(ws), ws_bytes, stream(), ctypes.c_void_p(fork[1].cuda_stream))
    _wgrad_joined((ws,), (dgamma, dbeta, dabias))
    return ga, dabias, gx0, dgamma, dbeta


def _ln_out(a, rows):
    """Output buffers of a fused post-norm over a's shape: x f32, xb bf16, mean, rstd."""
    dev = a.device
    return (torch.empty(a.shape, device=dev, dtype=torch.float32), torch.empty(a.shape, device=dev, dtype=torch.bfloat16),
            torch.empty(rows, device=dev, dtype=torch.float32), torch.empty(rows, device=dev, dtype=torch.float32))


class LinearLNFn(torch.autograd.Function):
    """(x, xb) = LayerNormResidual(LinearFn(inp, W), abias, x0, ...) with the norm in the GEMM's
    epilogue (hvk_linear_ln_fwd; C = 96: the stage-0 proj and the patch embedding on the skinny
    kernel; C = 192: the stage-1 proj and the stage-0 -> 1 PatchMerging on the 128 x 192 tile): one
    kernel forward instead of two with the same a / x / xb / mean / rstd bits; backward = the
    LayerNorm backward, then the Linear's (input grad + weight grad, the proj's xshift included)."""

    @staticmethod
    def forward(ctx, inp, weight, xshift, abias, x0, gamma, beta, sample_scale, rows_per_sample, eps):
        ctx.ln_leaves = (abias, gamma, beta)
        note_leaf_uses(_flat(ctx.ln_leaves), ctx)
        xin = _bf16(inp)
        wb, wt = _bf16_weight(weight)
        N, K = wb.shape
        M = xin.numel() // K
        a = torch.empty((*xin.shape[:-1], N), device=xin.device, dtype=torch.bfloat16)
        x, xb, mean, rstd = _ln_out(a, M)
        gamma, beta = _f32(gamma), _f32(beta)
        abias = _f32(abias) if abias is not None else None
        x0 = _f32(x0) if x0 is not None else None
        sample_scale = _f32(sample_scale) if sample_scale is not None else None
        call("hvk_linear_ln_fwd", ptr(xin), ptr(wb), M, K, N, ptr(abias), ptr(x0), ptr(gamma), ptr(beta),
             ptr(sample_scale), rows_per_sample, float(eps), ptr(a), ptr(x), ptr(xb), ptr(mean), ptr(rstd),
             stream())
        ctx.save_for_backward(xin, wb, a, abias, gamma, sample_scale, mean, rstd)
        ctx.wt = wt
        ctx.leaves = (weight,)
        note_leaf_uses(_flat(ctx.leaves), ctx)
        ctx.xshift = xshift.detach() if xshift is not None else None
        ctx.has_x0 = x0 is not None
        ctx.rps = rows_per_sample
        ctx.set_materialize_grads(False)
        return x, xb

    @staticmethod
    def backward(ctx, gx, gxb):
        xin, wb, a, abias, gamma, sample_scale, mean, rstd = ctx.saved_tensors
        r = _ln_residual_bwd(a, abias, gamma, sample_scale, mean, rstd, ctx.rps, ctx.has_x0, gx, gxb, ctx.ln_leaves)
        if r is None:
            return (None,) * 10
        ga, dabias, gx0, dgamma, dbeta = r
        N, K = wb.shape
        g2 = ga.reshape(-1, N)
        gin = None
        if ctx.needs_input_grad[0]:
            gin = (mm_nt(g2, _bf16_t(wb, ctx.wt)) if _native_nt(g2.shape[0], N, K)
                   else _dgrad_fallback(g2, wb)).reshape(xin.shape)
        dw = (weight_grad(g2, xin.reshape(-1, K), False, xshift=ctx.xshift, leaves=ctx.leaves)[0]
              if ctx.needs_input_grad[1] else None)
        return gin, dw, None, dabias, gx0, dgamma, dbeta, None, None, None


def linear_ln_supported(M, K, N):
    """The fused Linear + post-norm (hvk_linear_ln_fwd) is built for this shape and enabled
    (options.ln_epilogue; the C = 192 tile form also options.ln_epilogue_tile)."""
    return (OPTIONS.ln_epilogue and (N == 96 or OPTIONS.ln_epilogue_tile)
            and bool(_lib.load().hvk_linear_ln_supported(M, K, N)))


def linear_ln(inp, weight, x0, gamma, beta, sample_scale=None, rows_per_sample=1, eps=1e-5, abias=None,
              xshift=None):
    """LayerNormResidual(F.linear(inp, weight), x0, ...) with the norm fused into the GEMM's
    epilogue (callers check linear_ln_supported); xshift as for linear()."""
    return LinearLNFn.apply(inp, weight, xshift, abias, x0, gamma, beta, sample_scale, rows_per_sample, eps)


def layer_norm_residual(a, x0, gamma, beta, sample_scale=None, rows_per_sample=1, eps=1e-5,
                        abias=None):
    return LayerNormResidual.apply(a, abias, x0, gamma, beta, sample_scale, rows_per_sample, eps)


# --------------------------------------------------------------------------- MLP activation
class NormPool(torch.autograd.Function):
    """mean over tokens of LayerNorm(x) for the f32 stream x [B, T, C] (the final norm and
    the average pool, swinv2.py:833-835) as one kernel each way (hvk_ln_pool_fwd / _bwd)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, eps):
        note_leaf_uses((gamma, beta), ctx)
        x = _f32(x)
        B, T, C = x.shape
        dev = x.device
        y = torch.empty((B, C), device=dev, dtype=torch.float32)
        xsum = torch.empty_like(y)
        mean = torch.empty(B * T, device=dev, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        dg = torch.empty(C, device=dev, dtype=torch.float32)  # zeroed by the launch
        db = torch.empty_like(dg)
        call("hvk_ln_pool_fwd", ptr(x), ptr(_f32(gamma)), ptr(_f32(beta)), B, T, C, float(eps), ptr(y),
             ptr(xsum), ptr(mean), ptr(rstd), ptr(dg), ptr(db), stream())
        ctx.save_for_backward(x, gamma, mean, rstd, xsum)
        ctx.acc = (dg, db)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gamma, mean, rstd, xsum = ctx.saved_tensors
        dg, db = ctx.acc
        ctx.acc = None  # returned below as the only references: AccumulateGrad steals them
        B, T, C = x.shape
        dx = torch.empty_like(x)
        call("hvk_ln_pool_bwd", ptr(x), ptr(_f32(gamma)), ptr(mean), ptr(rstd), ptr(xsum),
             ptr(_f32(dy)), B, T, C, ptr(dx), ptr(dg), ptr(db), stream())
        return dx, dg, db, None


def norm_pool(x, gamma, beta, eps):
    return NormPool.apply(x, gamma, beta, eps)


class BiasGelu(torch.autograd.Function):
    """y = GELU(h + b) (exact erf form); backward also returns db (column sums)."""

    @staticmethod
    def forward(ctx, h, bias):
        h = _bf16(h)
        N = h.shape[-1]
        rows = h.numel() // N
        bias = _f32(bias) if bias is not None else None
        y = torch.empty_like(h)
        call("hvk_bias_gelu_fwd", ptr(h), ptr(bias), ptr(y), rows, N, stream())
        ctx.save_for_backward(h, bias)
        return y

    @staticmethod
    def backward(ctx, gy):
        h, bias = ctx.saved_tensors
        N = h.shape[-1]
        rows = h.numel() // N
        gy = _bf16(gy)
        gh = torch.empty_like(h)
        db = torch.empty(N, device=h.device, dtype=torch.float32) if bias is not None else None
        ws_bytes = _lib.load().hvk_bias_gelu_bwd_workspace_bytes(N)
        ws = torch.empty(ws_bytes // 4, device=h.device, dtype=torch.float32)
        call("hvk_bias_gelu_bwd", ptr(h), ptr(bias), ptr(gy), ptr(gh), ptr(db), ptr(ws), ws_bytes,
             rows, N, stream())
        return gh, db


def bias_gelu(h, bias):
    return BiasGelu.apply(h, bias)


class LinearGelu(torch.autograd.Function):
    """y = GELU(x W^T + b) as ONE kernel (gelu_fwd: fc1 GEMM with the bias + GELU epilogue,
    writing the bf16 pre-activation h for the backward); backward = the activation backward on
    h (db = its column sums) + the Linear backward."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        xb = _bf16(x)
        wb, wt = _bf16_weight(weight)
        N, K = wb.shape
        h, y = gelu_fwd(xb.reshape(-1, K), wb, bias)
        ctx.save_for_backward(xb, wb, h)
        ctx.wt = wt
        ctx.leaves = (weight,)
        note_leaf_uses(_flat(ctx.leaves), ctx)
        return y.reshape(*xb.shape[:-1], N)

    @staticmethod
    def backward(ctx, gy):
        xb, wb, h = ctx.saved_tensors
        N, K = wb.shape
        g2 = _bf16(gy).reshape(-1, N)
        M = g2.shape[0]
        gh = torch.empty_like(h)
        db = torch.empty(N, device=h.device, dtype=torch.float32)
        ws_bytes = _lib.load().hvk_bias_gelu_bwd_workspace_bytes(N)
        ws = torch.empty(ws_bytes // 4, device=h.device, dtype=torch.float32)
        call("hvk_bias_gelu_bwd", ptr(h), None, ptr(g2), ptr(gh), ptr(db), ptr(ws), ws_bytes, M, N,
             stream())
        gx = None
        if ctx.needs_input_grad[0]:
            gx = (mm_nt(gh, _bf16_t(wb, ctx.wt)) if _native_nt(M, N, K)
                  else _dgrad_fallback(gh, wb)).reshape(xb.shape)
        dw = weight_grad(gh, xb.reshape(-1, K), leaves=ctx.leaves)[0] if ctx.needs_input_grad[1] else None
        return gx, dw, db


def linear_gelu(x, weight, bias):
    """GELU(F.linear(x, weight, bias)): fused kernel where built, else GEMM + activation kernel."""
    N, K = weight.shape
    M = x.numel() // K
    if bias is not None and (((K in (96, 192) or K in _skinny_first_k())
                              and _lib.load().hvk_linear_gelu_supported(M, K, N)) or _tile_any(M, K, N)):
        return LinearGelu.apply(x, weight, bias)
    return bias_gelu(linear(x, weight), bias)


class MlpFn(torch.autograd.Function):
    """fc2(GELU(fc1(x))) (swinv2.py:58-65 with drop = 0): forward = the fused fc1 + GELU kernel
    and the fc2 GEMM; backward runs fc2's input gradient and the activation backward as ONE
    kernel (hvk_linear_gelu_bwd; the tiled hvk_gemm_gelu_bwd for stage 2) instead of GEMM ->
    bf16 dy1 -> activation kernel, and the fc1 bias gradient rides on fc1's weight-gradient
    kernel.  fc2's bias, when given, is added by the GEMM (else folded downstream)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        xb = _bf16(x)
        w1b, w1t = _bf16_weight(w1)
        w2b, w2t = _bf16_weight(w2)
        ctx.wts = (w1t, w2t)
        N1, K = w1b.shape
        N2 = w2b.shape[0]
        x2 = xb.reshape(-1, K)
        M = x2.shape[0]
        ctx.recompute = _gelu_recompute(M, K, N1, N2)
        if ctx.recompute:
            # GELU(h) is never stored: fc2 and its weight gradient recompute it per fragment
            h = mm_nt(x2, w1b, b1)
            y = torch.empty((M, N2), device=x2.device, dtype=torch.bfloat16)
            b = _f32(b2) if b2 is not None else None
            call("hvk_linear_gelu_in_fwd", ptr(h), ptr(w2b), ptr(b) if b is not None else None, ptr(y), M,
                 N1, N2, stream())
            ctx.save_for_backward(xb, w1b, w2b, h)
        elif OPTIONS.mlp_fused and _lib.load().hvk_mlp_fwd_supported(M, K, N1, N2):
            # stage-0 width: fc1 + GELU + fc2 in one kernel (no re-read of GELU(h))
            h = torch.empty((M, N1), device=x2.device, dtype=torch.bfloat16)
            y1 = torch.empty_like(h)
            y = torch.empty((M, N2), device=x2.device, dtype=torch.bfloat16)
            b = _f32(b2) if b2 is not None else None
            call("hvk_mlp_fwd", ptr(x2), ptr(w1b), ptr(_f32(b1)), ptr(w2b), ptr(b) if b is not None else None,
                 ptr(h), ptr(y1), ptr(y), M, K, N1, N2, stream())
            ctx.save_for_backward(xb, w1b, w2b, h, y1)
        else:
            h, y1 = gelu_fwd(x2, w1b, b1)
            y = mm_nt(y1, w2b, b2)
            ctx.save_for_backward(xb, w1b, w2b, h, y1)
        ctx.has_b2 = b2 is not None
        ctx.leaves = ((w1, b1), (w2, b2))
        note_leaf_uses(_flat(ctx.leaves), ctx)
        return y.reshape(*xb.shape[:-1], N2)

    @staticmethod
    def backward(ctx, gy):
        if ctx.recompute:
            xb, w1b, w2b, h = ctx.saved_tensors
        else:
            xb, w1b, w2b, h, y1 = ctx.saved_tensors
        N1, K = w1b.shape
        N2 = w2b.shape[0]
        g2 = _bf16(gy).reshape(-1, N2)
        M = g2.shape[0]
        if ctx.recompute:
            dw2, db2 = weight_grad(g2, h, ctx.has_b2, gelu_x=True, leaves=ctx.leaves[1])
        else:
            dw2, db2 = weight_grad(g2, y1, ctx.has_b2, leaves=ctx.leaves[1])
        gh = torch.empty_like(h)
        w2t = _bf16_t(w2b, ctx.wts[1])
        if (OPTIONS.mlp_fused and ctx.needs_input_grad[0] and not ctx.recompute
                and _lib.load().hvk_mlp_bwd_supported(M, N2, N1, K)):
            # stage-0 width: fc2's input gradient through GELU' and fc1's input gradient in one
            # kernel (gh stored for fc1's weight gradient, not re-read for gx)
            gx = torch.empty((M, K), device=h.device, dtype=torch.bfloat16)
            call("hvk_mlp_bwd", ptr(g2), ptr(w2t), ptr(h), ptr(_bf16_t(w1b, ctx.wts[0])), ptr(gh), ptr(gx),
                 M, N2, N1, K, stream())
            dw1, db1 = weight_grad(gh, xb.reshape(-1, K), True, leaves=ctx.leaves[0])  # fc1 bias gradient fused
            return gx.reshape(xb.shape), dw1, db1, dw2, db2
        lib = _lib.load()
        if ((_tile_ok(M, N2, N1) and not (N2 in _skinny_first_k() and lib.hvk_linear_gelu_bwd_supported(M, N2, N1)))
                or not lib.hvk_linear_gelu_bwd_supported(M, N2, N1)):
            call("hvk_gemm_gelu_bwd", ptr(g2), ptr(w2t), ptr(h), ptr(gh), M, N2, N1, stream())
        else:
            call("hvk_linear_gelu_bwd", ptr(g2), ptr(w2t), ptr(h), ptr(gh), None, M, N2, N1,
                 stream())
        gx = None
        if ctx.needs_input_grad[0]:
            gx = (mm_nt(gh, _bf16_t(w1b, ctx.wts[0])) if _native_nt(M, N1, K)
                  else _dgrad_fallback(gh, w1b)).reshape(xb.shape)
        dw1, db1 = weight_grad(gh, xb.reshape(-1, K), True, leaves=ctx.leaves[0])  # fc1 bias gradient fused
        return gx, dw1, db1, dw2, db2


class MlpLNFn(torch.autograd.Function):
    """(x, xb) = LayerNormResidual(fc2(GELU(fc1(inp))), abias = fc2's bias, x0, ...).  Stage-0
    width: ONE kernel forward (hvk_mlp_ln_fwd: the fused MLP with the block's norm2 in its
    epilogue, bit-identical to hvk_mlp_fwd + hvk_ln_residual_fwd).  Stage-1 width (N2 = 192):
    fc1 + GELU as MlpFn's kernel, fc2 on the 128 x 192 tile with the norm in its epilogue
    (hvk_linear_ln_fwd).  Backward = the LayerNorm backward, then MlpFn's chain for the path taken
    (fc2's bias gradient is the norm's dabias)."""

    @staticmethod
    def forward(ctx, inp, w1, b1, w2, abias, x0, gamma, beta, sample_scale, rows_per_sample, eps):
        ctx.ln_leaves = (abias, gamma, beta)
        note_leaf_uses(_flat(ctx.ln_leaves), ctx)
        xin = _bf16(inp)
        w1b, w1t = _bf16_weight(w1)
        w2b, w2t = _bf16_weight(w2)
        N1, K = w1b.shape
        N2 = w2b.shape[0]
        x2 = xin.reshape(-1, K)
        M = x2.shape[0]
        a = torch.empty((*xin.shape[:-1], N2), device=xin.device, dtype=torch.bfloat16)
        x, xb, mean, rstd = _ln_out(a, M)
        gamma, beta = _f32(gamma), _f32(beta)
        abias = _f32(abias) if abias is not None else None
        x0 = _f32(x0) if x0 is not None else None
        sample_scale = _f32(sample_scale) if sample_scale is not None else None
        ln_args = (ptr(abias), ptr(x0), ptr(gamma), ptr(beta), ptr(sample_scale), rows_per_sample, float(eps))
        ctx.fused = bool(_lib.load().hvk_mlp_ln_supported(M, K, N1, N2))
        if ctx.fused:
            h = torch.empty((M, N1), device=x2.device, dtype=torch.bfloat16)
            y1 = torch.empty_like(h)
            call("hvk_mlp_ln_fwd", ptr(x2), ptr(w1b), ptr(_f32(b1)), ptr(w2b), ptr(h), ptr(y1), ptr(a), M, K, N1,
                 N2, *ln_args, ptr(x), ptr(xb), ptr(mean), ptr(rstd), stream())
        else:
            h, y1 = gelu_fwd(x2, w1b, b1)
            call("hvk_linear_ln_fwd", ptr(y1), ptr(w2b), M, N1, N2, *ln_args, ptr(a), ptr(x), ptr(xb), ptr(mean),
                 ptr(rstd), stream())
        ctx.save_for_backward(xin, w1b, w2b, h, y1, a, abias, gamma, sample_scale, mean, rstd)
        ctx.wts = (w1t, w2t)
        ctx.leaves = ((w1, b1), (w2,))
        note_leaf_uses(_flat(ctx.leaves), ctx)
        ctx.has_x0 = x0 is not None
        ctx.rps = rows_per_sample
        ctx.set_materialize_grads(False)
        return x, xb

    @staticmethod
    def backward(ctx, gx, gxb):
        xin, w1b, w2b, h, y1, a, abias, gamma, sample_scale, mean, rstd = ctx.saved_tensors
        r = _ln_residual_bwd(a, abias, gamma, sample_scale, mean, rstd, ctx.rps, ctx.has_x0, gx, gxb, ctx.ln_leaves)
        if r is None:
            return (None,) * 11
        ga, dabias, gx0, dgamma, dbeta = r
        bwd = _mlp_bwd if ctx.fused else _mlp_bwd_tiled
        gin, dw1, db1, dw2 = bwd(ga, xin, w1b, w2b, h, y1, ctx.wts, ctx.needs_input_grad[0], ctx.leaves)
        return gin, dw1, db1, dw2, dabias, gx0, dgamma, dbeta, None, None, None


def _mlp_bwd(gy, xb, w1b, w2b, h, y1, wts, want_x, leaves=((), ())):
    """MlpFn's backward at the stage-0 width (the fused hvk_mlp_bwd chain; fc2's bias gradient is
    the caller's): (gx, dW1, db1, dW2)."""
    N1, K = w1b.shape
    N2 = w2b.shape[0]
    g2 = _bf16(gy).reshape(-1, N2)
    M = g2.shape[0]
    dw2 = weight_grad(g2, y1, leaves=leaves[1])[0]
    gh = torch.empty_like(h)
    w2t = _bf16_t(w2b, wts[1])
    gx = None
    if want_x:
        gx = torch.empty((M, K), device=h.device, dtype=torch.bfloat16)
        call("hvk_mlp_bwd", ptr(g2), ptr(w2t), ptr(h), ptr(_bf16_t(w1b, wts[0])), ptr(gh), ptr(gx), M, N2, N1, K,
             stream())
        gx = gx.reshape(xb.shape)
    else:
        call("hvk_linear_gelu_bwd", ptr(g2), ptr(w2t), ptr(h), ptr(gh), None, M, N2, N1, stream())
    dw1, db1 = weight_grad(gh, xb.reshape(-1, K), True, leaves=leaves[0])  # fc1 bias gradient fused
    return gx, dw1, db1, dw2


def _mlp_bwd_tiled(gy, xb, w1b, w2b, h, y1, wts, want_x, leaves=((), ())):
    """MlpFn's unfused backward chain (fc2's input gradient through GELU' as one kernel, fc1's
    input gradient, both weight gradients; fc2's bias gradient is the caller's): (gx, dW1, db1,
    dW2)."""
    N1, K = w1b.shape
    N2 = w2b.shape[0]
    g2 = _bf16(gy).reshape(-1, N2)
    M = g2.shape[0]
    dw2 = weight_grad(g2, y1, leaves=leaves[1])[0]
    gh = torch.empty_like(h)
    w2t = _bf16_t(w2b, wts[1])
    lib = _lib.load()
    if ((_tile_ok(M, N2, N1) and not (N2 in _skinny_first_k() and lib.hvk_linear_gelu_bwd_supported(M, N2, N1)))
            or not lib.hvk_linear_gelu_bwd_supported(M, N2, N1)):
        call("hvk_gemm_gelu_bwd", ptr(g2), ptr(w2t), ptr(h), ptr(gh), M, N2, N1, stream())
    else:
        call("hvk_linear_gelu_bwd", ptr(g2), ptr(w2t), ptr(h), ptr(gh), None, M, N2, N1, stream())
    gx = None
    if want_x:
        gx = (mm_nt(gh, _bf16_t(w1b, wts[0])) if _native_nt(M, N1, K)
              else _dgrad_fallback(gh, w1b)).reshape(xb.shape)
    dw1, db1 = weight_grad(gh, xb.reshape(-1, K), True, leaves=leaves[0])  # fc1 bias gradient fused
    return gx, dw1, db1, dw2


def mlp_ln_supported(M, K, N1, N2):
    """MlpLNFn applies: the fused stage-0 MLP + post-norm (hvk_mlp_ln_fwd and its fused backward
    chain), or fc1 + GELU on MlpFn's kernels with fc2 + post-norm on the tile's LN epilogue."""
    if not OPTIONS.ln_epilogue:
        return False
    lib = _lib.load()
    if OPTIONS.mlp_fused and lib.hvk_mlp_ln_supported(M, K, N1, N2) and lib.hvk_mlp_bwd_supported(M, N2, N1, K):
        return True
    return (N2 != 96 and linear_ln_supported(M, N1, N2) and not _gelu_recompute(M, K, N1, N2)
            and (((K in _gelu_skinny_k() or K in _skinny_first_k()) and lib.hvk_linear_gelu_supported(M, K, N1))
                 or _tile_any(M, K, N1))
            and (lib.hvk_linear_gelu_bwd_supported(M, N2, N1) or _tile_any(M, N2, N1)))


def mlp_ln(x, w1, b1, w2, x0, gamma, beta, sample_scale=None, rows_per_sample=1, eps=1e-5, abias=None):
    """LayerNormResidual(fc2(GELU(fc1(x))), x0, ...) with fc2's bias as the norm's abias, one kernel
    forward (callers check mlp_ln_supported)."""
    return MlpLNFn.apply(x, w1, b1, w2, abias, x0, gamma, beta, sample_scale, rows_per_sample, eps)


def mlp(x, w1, b1, w2, b2=None):
    """fc2(GELU(fc1(x))): the fused forward/backward kernels where built (skinny for stage 0-1,
    tiled for stage 2-3), else linear_gelu + linear."""
    N1, K = w1.shape
    M = x.numel() // K
    lib = _lib.load()
    if (b1 is not None and (((K in (96, 192) or K in _skinny_first_k()) and lib.hvk_linear_gelu_supported(M, K, N1))
                            or _tile_any(M, K, N1))
            and (lib.hvk_linear_gelu_bwd_supported(M, w2.shape[0], N1) or _tile_any(M, w2.shape[0], N1))):
        return MlpFn.apply(x, w1, b1, w2, b2)
    return linear(linear_gelu(x, w1, b1), w2, b2)


# --------------------------------------------------------------------------- PatchMerging
class PatchMergeGather(torch.autograd.Function):
    """[B, H*W, C] -> [B, H/2*W/2, 4C] in the concat order of swinv2.py:486-490."""

    @staticmethod
    def forward(ctx, x, H, W):
        B, L, C = x.shape
        x = _bf16(x)
        out = torch.empty((B, L // 4, 4 * C), device=x.device, dtype=torch.bfloat16)
        call("hvk_patch_merge_gather", ptr(x), ptr(out), B, H, W, C, stream())
        ctx.geom = (B, H, W, C)
        return out

    @staticmethod
    def backward(ctx, g):
        B, H, W, C = ctx.geom
        g = _bf16(g)
        gx = torch.empty((B, H * W, C), device=g.device, dtype=torch.bfloat16)
        call("hvk_patch_merge_scatter", ptr(g), ptr(gx), B, H, W, C, stream())
        return gx, None, None


def patchify_bf16(x, patch):
    """f32 images [B, C, H, W] -> bf16 token-major patches [B, (H/p)(W/p), C p p] in the
    Conv2d weight's (c, py, px) order: x.to(bfloat16) + permute + reshape in one kernel
    (swinv2.py:652-660).  Images carry no gradient; with one, or another patch size / channel
    count, the caller keeps the torch form."""
    B, C, H, W = x.shape
    out = torch.empty((B, (H // patch) * (W // patch), C * patch * patch), device=x.device,
                      dtype=torch.bfloat16)
    call("hvk_patchify_bf16", ptr(x.contiguous()), ptr(out), B, C, H, W, stream())
    return out


def patchify_u8_bf16(x, patch, mean, std):
    """uint8 images [B, 3, H, W] -> bf16 token-major patches with the device-side
    NormalizationFn (data.py:130-136) fused in: bf16((x - mean[c]) / std[c]) in the Conv2d
    weight's (c, py, px) order, one kernel (hvk_patchify_u8_bf16).  mean / std: f32 [3]."""
    B, C, H, W = x.shape
    if x.dtype != torch.uint8:
        raise TypeError("patchify_u8_bf16 takes uint8 images")
    out = torch.empty((B, (H // patch) * (W // patch), C * patch * patch), device=x.device,
                      dtype=torch.bfloat16)
    call("hvk_patchify_u8_bf16", ptr(x.contiguous()), ptr(out), ptr(_f32(mean)), ptr(_f32(std)), B, C, H, W,
         stream())
    return out


def normalize_u8(x, mean, std):
    """composer NormalizationFn on the device: f32 (x - mean[c]) / std[c] for uint8 [B, C, H, W]
    (hvk_normalize_u8)."""
    B, C, H, W = x.shape
    if x.dtype != torch.uint8:
        raise TypeError("normalize_u8 takes uint8 images")
    out = torch.empty((B, C, H, W), device=x.device, dtype=torch.float32)
    call("hvk_normalize_u8", ptr(x.contiguous()), ptr(out), ptr(_f32(mean)), ptr(_f32(std)), B, C, H * W,
         stream())
    return out


def patch_merge_gather(x, H, W):
    return PatchMergeGather.apply(x, H, W)


def merge_linear_supported(B, H, W, C, N):
    """PatchMerging's gather folded into its reduction GEMM both ways (hvk_merge_*; option
    merge_gemm) for x [B, H*W, C] and the Linear 4C -> N."""
    if not OPTIONS.merge_gemm:
        return False
    lib = _lib.load()
    return bool(lib.hvk_merge_gemm_supported(B, H, W, C, N) and lib.hvk_merge_weight_grad_supported(B, H, W, C, N))


def merge_linear_ln_supported(B, H, W, C, N):
    """... and with PatchMerging's norm in the GEMM epilogue (N = 192; options ln_epilogue,
    ln_epilogue_tile)."""
    return (merge_linear_supported(B, H, W, C, N) and OPTIONS.ln_epilogue and OPTIONS.ln_epilogue_tile
            and bool(_lib.load().hvk_merge_linear_ln_supported(B, H, W, C, N)))


def _merge_linear_bwd(ctx, xb, wb, ga):
    """Input gradient (scattered to the token rows) and weight gradient (gathering on its DMA) of
    PatchMerging's reduction Linear for the output gradient ga [M, N] bf16."""
    B, H, W, C, N = ctx.geo
    ga = _bf16(ga).contiguous()
    gx = dw = None
    if ctx.needs_input_grad[0]:
        gx = torch.empty((B, H * W, C), device=ga.device, dtype=torch.bfloat16)
        call("hvk_merge_gemm_dgrad", ptr(ga), ptr(_bf16_t(wb, ctx.wt)), ptr(gx), B, H, W, C, N, stream())
    if ctx.needs_input_grad[1]:
        lib = _lib.load()
        M = B * H * W // 4
        nb = lib.hvk_weight_grad_workspace(M, N, 4 * C)
        ws = torch.empty(nb // 4, device=ga.device, dtype=torch.float32)
        dw = torch.empty((N, 4 * C), device=ga.device, dtype=torch.float32)
        fork = _wgrad_fork(ctx.leaves)  # options.wgrad_stream: on the weight-gradient side stream
        with torch.cuda.stream(fork[1]) if fork else contextlib.nullcontext():
            call("hvk_merge_weight_grad", ptr(ga), ptr(xb), ptr(dw), B, H, W, C, N, ptr(ws), nb, stream())
        if fork:
            _wgrad_joined((ga, xb, ws), (dw,))
            _wgrad_outputs(dw)
    return gx, dw


class MergeLinearFn(torch.autograd.Function):
    """PatchMerging's strided gather + reduction Linear (swinv2.py:484-494) as one GEMM each way:
    forward hvk_merge_gemm_fwd (the gather on the operand loads), backward hvk_merge_gemm_dgrad
    (the input gradient scattered by the GEMM's store) and hvk_merge_weight_grad; the same bits
    as patch_merge_gather + linear, without the [T/4, 4C] tensor."""

    @staticmethod
    def forward(ctx, x, weight, H, W):
        xb = _bf16(x).contiguous()
        wb, wt = _bf16_weight(weight)
        B, L, C = xb.shape
        N = wb.shape[0]
        y = torch.empty((B, L // 4, N), device=xb.device, dtype=torch.bfloat16)
        call("hvk_merge_gemm_fwd", ptr(xb), ptr(wb), ptr(y), B, H, W, C, N, stream())
        ctx.save_for_backward(xb, wb)
        ctx.wt = wt
        ctx.geo = (B, H, W, C, N)
        ctx.leaves = (weight,)
        note_leaf_uses(_flat(ctx.leaves), ctx)
        return y

    @staticmethod
    def backward(ctx, gy):
        xb, wb = ctx.saved_tensors
        gx, dw = _merge_linear_bwd(ctx, xb, wb, gy.reshape(-1, ctx.geo[4]))
        return gx, dw, None, None


class MergeLinearLNFn(torch.autograd.Function):
    """MergeLinearFn with PatchMerging's norm in the GEMM epilogue (hvk_merge_linear_ln_fwd, N =
    192: the stage-0 -> 1 merge): (x, xb) as linear_ln(patch_merge_gather(x), ...) bit for bit;
    backward = the norm's, then MergeLinearFn's."""

    @staticmethod
    def forward(ctx, x, weight, gamma, beta, eps, H, W):
        ctx.ln_leaves = (gamma, beta)
        note_leaf_uses(_flat(ctx.ln_leaves), ctx)
        xb = _bf16(x).contiguous()
        wb, wt = _bf16_weight(weight)
        B, L, C = xb.shape
        N = wb.shape[0]
        M = B * L // 4
        a = torch.empty((B, L // 4, N), device=xb.device, dtype=torch.bfloat16)
        xo, xob, mean, rstd = _ln_out(a, M)
        gamma, beta = _f32(gamma), _f32(beta)
        call("hvk_merge_linear_ln_fwd", ptr(xb), ptr(wb), B, H, W, C, N, ptr(gamma), ptr(beta), float(eps), ptr(a),
             ptr(xo), ptr(xob), ptr(mean), ptr(rstd), stream())
        ctx.save_for_backward(xb, wb, a, gamma, mean, rstd)
        ctx.wt = wt
        ctx.geo = (B, H, W, C, N)
        ctx.leaves = (weight,)
        note_leaf_uses(_flat(ctx.leaves), ctx)
        ctx.set_materialize_grads(False)
        return xo, xob

    @staticmethod
    def backward(ctx, gx, gxb):
        xb, wb, a, gamma, mean, rstd = ctx.saved_tensors
        r = _ln_residual_bwd(a, None, gamma, None, mean, rstd, 1, False, gx, gxb, ctx.ln_leaves)
        if r is None:
            return (None,) * 7
        ga, _, _, dgamma, dbeta = r
        gin, dw = _merge_linear_bwd(ctx, xb, wb, ga.reshape(-1, ctx.geo[4]))
        return gin, dw, dgamma, dbeta, None, None, None


def merge_linear(x, weight, H, W):
    """F.linear(patch_merge_gather(x, H, W), weight) as one GEMM each way (callers check
    merge_linear_supported)."""
    return MergeLinearFn.apply(x, weight, H, W)


def merge_linear_ln(x, weight, gamma, beta, eps, H, W):
    """linear_ln(patch_merge_gather(x, H, W), weight, None, gamma, beta, eps=eps) with the gather
    in the GEMM (callers check merge_linear_ln_supported)."""
    return MergeLinearLNFn.apply(x, weight, gamma, beta, eps, H, W)


# --------------------------------------------------------------------------- losses
class MultitaskCE(torch.autograd.Function):
    """sum_h coeff[h] * mean_b CE(logits[:, off[h]:off[h+1]], target_h)."""

    @staticmethod
    def forward(ctx, logits, head_off, coeff, targets, soft):
        logits = _f32(logits)
        B, ld = logits.shape
        nh = head_off.numel() - 1
        row_loss = torch.empty((nh, B), device=logits.device, dtype=torch.float32)
        lse = torch.empty((nh, B), device=logits.device, dtype=torch.float32)
        call("hvk_multitask_ce_fwd", ptr(logits), ld, B, nh, ptr(head_off), ptr(targets),
             ptr(soft), ptr(row_loss), ptr(lse), stream())
        ctx.save_for_backward(logits, head_off, coeff, targets, soft, lse)
        return (row_loss.mean(dim=1) * coeff).sum()

    @staticmethod
    def backward(ctx, gout):
        logits, head_off, coeff, targets, soft, lse = ctx.saved_tensors
        B, ld = logits.shape
        nh = head_off.numel() - 1
        dlogits = torch.empty_like(logits)
        gout = _f32(gout.reshape(1))
        call("hvk_multitask_ce_bwd", ptr(logits), ld, B, nh, ptr(head_off), ptr(targets),
             ptr(soft), ptr(lse), ptr(coeff), ptr(gout), ptr(dlogits), stream())
        return dlogits, None, None, None, None


def multitask_cross_entropy(logits, head_off, coeff, targets=None, soft=None):
    if (targets is None) == (soft is None):
        raise ValueError("exactly one of hard targets / soft targets")
    if targets is not None:
        targets = targets.to(torch.int64).contiguous()
    if soft is not None:
        soft = _f32(soft)
    return MultitaskCE.apply(logits, head_off, coeff, targets, soft)


class HierarchicalCE(torch.autograd.Function):
    """HXE over leaf logits [B, L]; see include/hvk.h for the definition."""

    @staticmethod
    def forward(ctx, logits, targets, perm, node_start, node_end, tier_base, level_coeff):
        logits = _f32(logits)
        B, L = logits.shape
        row_loss = torch.empty(B, device=logits.device, dtype=torch.float32)
        lse = torch.empty((B, 8), device=logits.device, dtype=torch.float32)
        call("hvk_hxe_fwd", ptr(logits), B, L, ptr(perm), ptr(targets), ptr(node_start),
             ptr(node_end), ptr(tier_base), ptr(level_coeff), ptr(row_loss), ptr(lse), stream())
        ctx.save_for_backward(logits, targets, perm, node_start, node_end, tier_base,
                              level_coeff, lse)
        ctx.has_perm = perm is not None
        return row_loss.mean()

    @staticmethod
    def backward(ctx, gout):
        logits, targets, perm, node_start, node_end, tier_base, level_coeff, lse = ctx.saved_tensors
        B, L = logits.shape
        dlogits = torch.empty_like(logits)
        gout = _f32(gout.reshape(1))
        call("hvk_hxe_bwd", ptr(logits), B, L, ptr(perm if ctx.has_perm else None), ptr(targets),
             ptr(node_start), ptr(node_end), ptr(tier_base), ptr(level_coeff), ptr(lse),
             ptr(gout), ptr(dlogits), stream())
        return dlogits, None, None, None, None, None, None


def hierarchical_cross_entropy(logits, targets, perm, node_start, node_end, tier_base, level_coeff):
    return HierarchicalCE.apply(logits, targets.to(torch.int64).contiguous(), perm, node_start,
                                node_end, tier_base, level_coeff)
