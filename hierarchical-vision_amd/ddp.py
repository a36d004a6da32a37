"""Data-parallel gradient exchange: bucketed all-reduce over RCCL, overlapped with
the backward pass (the one hot-path collective; the reference
gets it implicitly from composer's DDP wrapper, main.py:104-124).

Design for MI355X:
* Gradients live in a few large flat f32 buffers ("buckets"), one per ~`bucket_mb`
  of parameters in reverse registration order (= roughly backward order); every
  ``param.grad`` is a view into its bucket, so there is no pack / unpack copy.
* A post-accumulate-grad hook counts arrivals; when a bucket's last gradient is
  accumulated the bucket's all-reduce is enqueued immediately (RCCL runs it on
  its own HIP stream, ordered after the producing kernels), so communication of
  late layers overlaps the backward of early ones.  Buckets are big (default
  64 MB): xGMI is point-to-point (7 links/GPU) and RCCL's ring/tree per-call
  cost is amortised only by large messages.
* ``synchronize()`` waits for all buckets (makes the current stream wait on the
  RCCL stream, no host sync).  The 1/world mean is not a separate pass over the 141 MB: the
  trainer hands it to the fused optimizer step as a gradient scale (optim.DecoupledSGDW);
  ``synchronize(scale=True)`` divides in place for optimizers that cannot take it.
No other collective runs in the step.
"""
import torch
import torch.distributed as dist


class GradientBuckets:
    def __init__(self, module: torch.nn.Module, bucket_mb: float = 64.0, process_group=None):
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        params = [p for p in module.parameters() if p.requires_grad]
        self.params = params
        self.enabled = self.world > 1
        self.defer = False  # graph mode: no hook-launched all-reduce (allreduce_now() instead)
        self.buckets = []
        self._hooks = []
        if not self.enabled:  # single rank: nothing to exchange, let autograd own .grad
            return
        limit = int(bucket_mb * 1024 * 1024 / 4)
        self.buckets = []  # list of (flat buffer, [params])
        cur, size = [], 0
        for p in reversed(params):
            if cur and size + p.numel() > limit:
                self.buckets.append(self._make(cur, size))
                cur, size = [], 0
            cur.append(p)
            size += p.numel()
        if cur:
            self.buckets.append(self._make(cur, size))
        self._pending = [0] * len(self.buckets)
        self._works = [None] * len(self.buckets)
        for bi, (_, ps) in enumerate(self.buckets):
            for p in ps:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(bi)))
        self.reset()

    @staticmethod
    def _make(params, n):
        dev = params[0].device
        flat = torch.zeros(n, device=dev, dtype=torch.float32)
        off = 0
        for p in params:
            if p.dtype != torch.float32:
                raise TypeError("master parameters must be f32")
            p.grad = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        return flat, params

    def _make_hook(self, bi):
        def hook(p):
            self._pending[bi] -= 1
            if self._pending[bi] == 0 and self.enabled and not self.defer:
                flat = self.buckets[bi][0]
                self._works[bi] = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.pg,
                                                  async_op=True)
        return hook

    def reset(self):
        """Zero every bucket in place (grads stay views) before the next backward."""
        if not self.enabled:
            for p in self.params:
                p.grad = None
            return
        for i, (flat, ps) in enumerate(self.buckets):
            flat.zero_()
            self._pending[i] = len(ps)
            self._works[i] = None
            for p in ps:  # re-attach if an optimizer set .grad = None
                if p.grad is None or p.grad.data_ptr() < flat.data_ptr() or \
                        p.grad.data_ptr() >= flat.data_ptr() + flat.numel() * 4:
                    raise RuntimeError("param.grad was detached from its bucket; "
                                       "use zero_grad(set_to_none=False) or buckets.reset()")

    def synchronize(self, scale=True):
        """Wait for every bucket's all-reduce; with scale, turn the sums into means in place
        (scale=False leaves sums for an optimizer that applies 1/world itself)."""
        if not self.enabled:
            return
        for i, (flat, _) in enumerate(self.buckets):
            w = self._works[i]
            if w is None:  # a bucket whose grads never arrived (unused params): reduce now
                w = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
            w.wait()
            if scale:
                flat.div_(self.world)

    def zero_(self):
        """Zero the buckets in place (graph mode: captured at the start of the backward graph)."""
        for flat, _ in self.buckets:
            flat.zero_()

    def allreduce_now(self):
        """Graph mode: all-reduce every bucket (SUM) between the backward and optimizer graph
        replays, eagerly (RCCL is not captured); the mean is taken inside the optimizer graph."""
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
