"""Data-parallel gradient exchange: bucketed all-reduce over RCCL, overlapped with
the backward pass (the one hot-path collective; the reference
gets it implicitly from composer's DDP wrapper, main.py:104-124).

Design for MI355X:
* Gradients live in a few large flat f32 buffers ("buckets") in reverse registration order
  (= roughly backward order): the first closes as soon as it holds ``first_mb`` (so it is the
  head's gradients -- the first ready -- even when one of them alone is larger: the 30.7 MB
  10 000-leaf HXE head weight), the middle ones hold up to ``bucket_mb`` each, and the LAST holds
  only the earliest-registered ``last_mb`` (patch embedding, stage 0, ...): its all-reduce can
  start only when the backward's final gradient lands, so it is the exchange's exposed tail and
  is kept small; every larger bucket is enqueued while the backward still runs.  After the
  exchange every ``param.grad`` is a view into its bucket (the optimizer and the clip read the
  buckets, no pack / unpack copy).
* Between steps ``param.grad`` is None, so autograd hands each fresh weight gradient over
  without a ``grad += new`` pass (and the buckets need no per-step zero_); the
  post-accumulate-grad hook copies it into its bucket view (one read + one write of the
  gradient instead of zero + read-add-write) and counts arrivals: when a bucket's last
  gradient is in, the bucket's all-reduce is enqueued immediately (RCCL runs it on its
  own HIP stream, ordered after the producing kernels), so communication of late layers
  overlaps the backward of early ones.  Later buckets are big (default 64 MB): xGMI is
  point-to-point (7 links/GPU) and RCCL's ring/tree per-call cost is amortised only by
  large messages.
* ``synchronize()`` waits for all buckets (makes the current stream wait on the
  RCCL stream, no host sync).  The 1/world mean is not a separate pass over the 141 MB: the
  trainer hands it to the fused optimizer step as a gradient scale (optim.DecoupledSGDW);
  ``synchronize(scale=True)`` divides in place for optimizers that cannot take it.
No other collective runs in the step.
"""
import contextlib

import torch
import torch.distributed as dist

from . import ops


class GradientBuckets:
    def __init__(self, module: torch.nn.Module, bucket_mb: float = 64.0, process_group=None,
                 first_mb: float = 8.0, force: bool = False, last_mb: float = 4.0):
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        params = [p for p in module.parameters() if p.requires_grad]
        self.params = params
        # force: exchange even at world 1 (a one-rank RCCL group exercises the whole hook /
        # all-reduce / synchronize path on a one-GPU box, tests/test_gpu_ddp.py)
        self.enabled = self.world > 1 or (force and dist.is_initialized())
        self.defer = False  # graph mode: no hook-launched all-reduce (allreduce_now() instead)
        # grad_accum: microbatches before the last only accumulate into the bucket views (no
        # arrival count, no all-reduce: composer's DDP no_sync)
        self.accumulating = False
        # measurement only (Trainer.comm_timing, tools/ddp_trace.py): a list -> each bucket's
        # all-reduce enqueue is marked on the producing stream, (bucket, trainer._Mark) appended
        self.trace = None
        self.buckets = []
        self._hooks = []
        if not self.enabled:  # single rank: nothing to exchange, let autograd own .grad
            return
        self.buckets = []  # list of (flat buffer, [params])
        self._view = {}    # param -> its view in the bucket
        for group in self.plan([p.numel() for p in params], bucket_mb, first_mb, last_mb):
            ps = [params[i] for i in group]
            self.buckets.append(self._make(ps, sum(p.numel() for p in ps)))
        self._pending = [0] * len(self.buckets)
        self._works = [None] * len(self.buckets)
        for bi, (_, ps) in enumerate(self.buckets):
            for p in ps:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(bi)))
        self.reset()

    @staticmethod
    def plan(numels, bucket_mb=64.0, first_mb=8.0, last_mb=4.0):
        """Bucket assignment for parameters of `numels` elements (f32) in registration order:
        a list of buckets, each a list of parameter indices, in exchange (= backward) order.
        The tail -- the earliest-registered parameters, at least one, up to min(last_mb,
        bucket_mb) -- is the last bucket; the rest in reverse order: the first bucket closes
        once it reaches first_mb (a parameter larger than that joins it rather than waiting
        behind it), later ones are cut before they would exceed bucket_mb."""
        mb = 1024 * 1024 / 4
        limit, first = int(bucket_mb * mb), int(min(first_mb, bucket_mb) * mb)
        tail_cap = int(min(last_mb, bucket_mb) * mb)
        n_tail, t = 1, numels[0] if numels else 0
        while n_tail < len(numels) - 1 and t + numels[n_tail] <= tail_cap:
            t += numels[n_tail]
            n_tail += 1
        if len(numels) <= 1:
            n_tail = len(numels)
        out, cur, size = [], [], 0
        for i in range(len(numels) - 1, n_tail - 1, -1):
            if not out:  # first bucket: close once it has first_mb
                cur.append(i)
                size += numels[i]
                if size >= first:
                    out.append(cur)
                    cur, size = [], 0
                continue
            if cur and size + numels[i] > limit:
                out.append(cur)
                cur, size = [], 0
            cur.append(i)
            size += numels[i]
        if cur:
            out.append(cur)
        if n_tail:
            out.append(list(range(n_tail - 1, -1, -1)))
        return out

    def _make(self, params, n):
        dev = params[0].device
        flat = torch.zeros(n, device=dev, dtype=torch.float32)
        off = 0
        for p in params:
            if p.dtype != torch.float32:
                raise TypeError("master parameters must be f32")
            self._view[p] = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        return flat, params

    def _make_hook(self, bi):
        def hook(p):
            # a gradient computed on the weight-gradient side stream (ops.wgrad_stream_scope)
            # is copied, and its bucket's all-reduce issued, on that stream (after everything
            # the current stream queued so far): the hook does not make the backward wait
            side = ops.wgrad_side_pending() if p.is_cuda else None
            if side is not None and not ops.wgrad_produced_on_side(p.grad):
                side.wait_stream(torch.cuda.current_stream())  # a gradient the current stream wrote
            with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
                self._hook_body(bi, p, side)
        return hook

    def _hook_body(self, bi, p, side):
        v = self._view[p]
        if p.grad is not v:  # the fresh gradient autograd handed over -> its bucket slot
            g = p.grad
            v.copy_(g)
            if side is not None:
                ops.wgrad_hold(g)  # freed after the join (ops.wgrad_hold)
            p.grad = v
        if self.accumulating:  # later microbatches add onto the view in place
            return
        self._pending[bi] -= 1
        if self._pending[bi] == 0 and self.enabled and not self.defer:
            flat = self.buckets[bi][0]
            if self.trace is not None:  # the enqueue point on the producing stream (trainer._Mark)
                from .trainer import _Mark
                self.trace.append((bi, _Mark(p.is_cuda)))
            self._works[bi] = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.pg,
                                              async_op=True)

    def reset(self):
        """Before the next backward: every param.grad None (autograd hands the new gradient
        over; the hook copies it into the bucket), arrival counts re-armed.  No zero pass."""
        for p in self.params:
            p.grad = None
        if not self.enabled:
            return
        for i, (flat, ps) in enumerate(self.buckets):
            self._pending[i] = len(ps)
            self._works[i] = None

    def _fill_missing(self, i):
        """Parameters of bucket i that got no gradient this backward: zero slots."""
        for p in self.buckets[i][1]:
            v = self._view[p]
            if p.grad is not v:
                if p.grad is None:
                    v.zero_()
                else:
                    v.copy_(p.grad)
                p.grad = v

    def synchronize(self, scale=True):
        """Wait for every bucket's all-reduce; with scale, turn the sums into means in place
        (scale=False leaves sums for an optimizer that applies 1/world itself)."""
        if not self.enabled:
            return
        for i, (flat, _) in enumerate(self.buckets):
            w = self._works[i]
            if w is None:  # a bucket whose grads never all arrived (unused params): reduce now
                self._fill_missing(i)
                w = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
            w.wait()
            if scale:
                flat.div_(self.world)

    def zero_(self):
        """Zero the buckets in place (graph mode: captured at the start of the backward graph,
        which the gradients of that capture then overwrite or add to)."""
        for flat, _ in self.buckets:
            flat.zero_()

    def allreduce_now(self):
        """Graph mode: all-reduce every bucket (SUM) between the backward and optimizer graph
        replays, eagerly (RCCL is not captured); the mean is taken inside the optimizer graph."""
        for i in range(len(self.buckets)):
            self._fill_missing(i)
        works = [dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
                 for flat, _ in self.buckets]
        for w in works:
            w.wait()

    def scale_(self):
        for flat, _ in self.buckets:
            flat.div_(self.world)

    def flat_buffers(self):
        return [b[0] for b in self.buckets]

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
