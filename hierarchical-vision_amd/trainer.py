"""One training step with the event order composer.Trainer uses for the hot path
(SURVEY.md §3.2): forward -> BEFORE_LOSS -> loss -> AFTER_LOSS -> backward (with
bucketed RCCL all-reduce overlapped) -> AFTER_BACKWARD (clipping) -> optimizer
step -> BATCH_END (EMA).  bf16 autocast on the GPU; no host synchronisation
inside the step.

Graph mode (`capture()` / `replay()`): the step is hundreds of small launches, so on
MI355X it is host-bound when issued one by one from Python.  The forward + loss + backward
is captured once as a HIP graph (torch.cuda.CUDAGraph over hipGraph), the gradient mean +
clipping + optimizer update as a second one; a step is two graph replays with, for
world > 1, the bucketed RCCL all-reduce issued eagerly between them (RCCL is not captured).
The batch must live in the static tensors passed to capture() (copy new data into them).
BATCH_END algorithms (EMA: host-side counters) run eagerly after the replays."""
import time

import torch

from . import ops
from .algorithmic import Event, State
from .ddp import GradientBuckets
from .options import OPTIONS


def resolve_grad_accum(grad_accum, device_type):
    """composer's `grad_accum` as main.py passes it (main.py:38-41, :121): "auto" needs a GPU
    (the same ValueError on CPU) and resolves to 1 here -- composer's "auto" only shrinks the
    microbatch after a CUDA OOM, and a bs256 SwinV2 step uses a small part of 288 GB of HBM;
    otherwise a positive integer number of microbatches per batch."""
    if grad_accum == "auto":
        if device_type != "cuda":
            raise ValueError('grad_accum="auto" requires training with a GPU; please specify '
                             'grad_accum as an integer')
        return 1
    if isinstance(grad_accum, bool) or not isinstance(grad_accum, int) or grad_accum < 1:
        raise ValueError(f"grad_accum must be 'auto' or a positive integer, got {grad_accum!r}")
    return grad_accum


def _split_batch(batch, n):
    """The batch's tensors cut into n equal microbatches along dim 0 (composer's
    `_default_split_batch` for a tuple/list batch)."""
    size = batch[0].shape[0]
    if size % n:
        raise ValueError(f"batch of {size} samples does not split into grad_accum={n} "
                         "equal microbatches")
    return [type(batch)(t.narrow(0, i * (size // n), size // n) for t in batch)
            for i in range(n)]


class _Mark:
    """A point in the step's timeline: a timing event on the current HIP stream (CUDA), else the
    host clock (CPU / gloo tests, where the backward runs synchronously)."""

    def __init__(self, cuda):
        if cuda:
            self.ev = torch.cuda.Event(enable_timing=True)
            self.ev.record()
        else:
            self.ev, self.t = None, time.perf_counter()

    def ms_to(self, later):
        if self.ev is not None:
            return self.ev.elapsed_time(later.ev)
        return 1000.0 * (later.t - self.t)


def comm_report(records):
    """Exchange timing of the steps recorded with Trainer.comm_timing = [] (world > 1):
    exposed_ms = mean GPU time from the end of the backward to the point where the current stream
    has waited for every bucket's all-reduce (buckets.synchronize(); the exchange time the
    backward did not hide), backward_ms its mean length, and per bucket the mean enqueue offset
    before the end of the backward (ms; the overlap window each all-reduce had).  Synchronises."""
    if not records:
        return None
    if records[0]["bwd_start"].ev is not None:
        torch.cuda.synchronize()
    exposed = [r["bwd_end"].ms_to(r["sync_end"]) for r in records]
    bwd = [r["bwd_start"].ms_to(r["bwd_end"]) for r in records]
    nb = max(len(r["buckets"]) for r in records)
    offs = [[] for _ in range(nb)]
    for r in records:
        for bi, e in r["buckets"]:
            offs[bi].append(e.ms_to(r["bwd_end"]))
    return {"steps": len(records), "exposed_ms": round(sum(exposed) / len(exposed), 3),
            "exposed_ms_max": round(max(exposed), 3), "backward_ms": round(sum(bwd) / len(bwd), 3),
            "bucket_enqueue_before_bwd_end_ms": [round(sum(o) / len(o), 3) if o else None for o in offs]}


class Trainer:
    def __init__(self, model, optimizer, algorithms=(), bucket_mb=64.0, dtype=torch.bfloat16,
                 device_transforms=None, grad_accum=1):
        self.model = model
        self.optimizer = optimizer
        self.algorithms = list(algorithms)
        self.dtype = dtype
        # composer DataSpec device_transforms (data.py:154-164): applied to each batch on the
        # device; a NormalizationFn the model can absorb (data.NormalizationFn.fuse_into) is
        # folded into its patch gather once and costs no pass of its own
        self.device_transforms = device_transforms
        if device_transforms is not None and getattr(device_transforms, "fuse_into", None):
            if device_transforms.fuse_into(model):
                self.device_transforms = None
        self.state = State(model, optimizer)
        self.buckets = GradientBuckets(model, bucket_mb=bucket_mb)
        dev = next(model.parameters()).device.type
        self.grad_accum = resolve_grad_accum(grad_accum, dev)
        # a list -> each eager step appends its exchange timing events (comm_report); None: off
        self.comm_timing = None
        # eager steps the host may have enqueued ahead of the GPU (None: unbounded, the default;
        # bench.py --steps-in-flight).  The side stream's buffers no longer need it
        # (ops.wgrad_hold), and bounding the SwinV2-T step to 2 cost 1.5 %
        # (profiles/round6/inflight/).
        self.max_steps_in_flight = None
        self._in_flight = []
        self._run(Event.INIT)

    def _run(self, event):
        for a in self.algorithms:
            if a.match(event, self.state):
                a.apply(event, self.state, None)

    def train_step(self, batch):
        st = self.state
        if self.max_steps_in_flight and len(self._in_flight) >= self.max_steps_in_flight:
            self._in_flight.pop(0).synchronize()  # the step max_steps_in_flight back is done
        if self.device_transforms is not None:
            batch = self.device_transforms(batch)
        # every .grad None and the arrival counts re-armed before the backward: after a
        # capture()/replay() .grad still points at the graph's gradient tensors, which autograd
        # would otherwise accumulate this step's gradient onto
        self.buckets.reset()
        self.model.train()
        dev_type = batch[0].device.type
        micro = _split_batch(batch, self.grad_accum) if self.grad_accum > 1 else [batch]
        total = None
        for i, mb in enumerate(micro):
            # composer's microbatch loop: each microbatch's loss scaled by its share of the
            # batch, gradients accumulated; the all-reduce hooks fire on the last one only
            # (DDP no_sync for the others)
            self.buckets.accumulating = i < len(micro) - 1
            st.batch = mb
            ops.reset_leaf_uses()  # the side stream's per-parameter use counts start with this forward
            with torch.autocast(device_type=dev_type, dtype=self.dtype, enabled=dev_type == "cuda"):
                st.outputs = self.model(st.batch)
            self._run(Event.BEFORE_LOSS)
            st.loss = self.model.loss(st.outputs, st.batch)
            self._run(Event.AFTER_LOSS)
            if len(micro) > 1:
                st.loss = st.loss * (1.0 / len(micro))
            # single rank: parameter gradients may run on the weight-gradient side stream
            # (ops.wgrad_stream_scope; a parameter still holding a gradient, i.e. a later
            # microbatch, stays on this stream).  With the bucketed all-reduce only under
            # options.wgrad_stream_multi_rank: a bucket can only start once the side stream, which
            # runs behind, has produced it (the dp2 gloo rehearsal measured -8 %,
            # profiles/round5/wgrad_stream/dp2_ab.txt; RCCL over xGMI is unmeasured)
            side = dev_type == "cuda" and (not self.buckets.enabled or OPTIONS.wgrad_stream_multi_rank)
            timing = self.comm_timing is not None and self.buckets.enabled and i == len(micro) - 1
            if timing:
                ev = {"bwd_start": _Mark(dev_type == "cuda")}
                self.buckets.trace = []
            with ops.wgrad_stream_scope(side):
                st.loss.backward()
            if timing:
                ev["bwd_end"] = _Mark(dev_type == "cuda")
            total = st.loss.detach() if total is None else total + st.loss.detach()
        self.buckets.accumulating = False
        st.batch = batch
        st.loss = total
        self._grad_mean()
        if timing:
            ev["sync_end"] = _Mark(dev_type == "cuda")
            ev["buckets"], self.buckets.trace = self.buckets.trace, None
            self.comm_timing.append(ev)
        self._run(Event.AFTER_BACKWARD)
        self.optimizer.step()
        self.buckets.reset()
        st.timestamp_batch += 1
        self._run(Event.BATCH_END)
        if self.max_steps_in_flight and batch[0].device.type == "cuda":
            done = torch.cuda.Event()
            done.record()
            self._in_flight.append(done)
        return st.loss

    def _grad_mean(self, wait=True):
        """Bucket all-reduces done -> mean gradients: handed to the optimizer as a scale when it
        can fold it into its update (no extra pass), else divided in place."""
        fold = self.buckets.enabled and getattr(self.optimizer, "supports_grad_scale", lambda: False)()
        if wait:
            self.buckets.synchronize(scale=not fold)
        elif self.buckets.enabled and not fold:
            self.buckets.scale_()
        if fold:
            self.optimizer.pending_grad_scale = 1.0 / self.buckets.world

    # ---------------------------------------------------------------- graph mode
    def _forward_backward(self, batch):
        st = self.state
        if self.device_transforms is not None:
            batch = self.device_transforms(batch)
        st.batch = batch
        self.model.train()
        if self.buckets.enabled:
            self.buckets.zero_()
        with torch.autocast(device_type="cuda", dtype=self.dtype):
            st.outputs = self.model(st.batch)
        self._run(Event.BEFORE_LOSS)
        st.loss = self.model.loss(st.outputs, st.batch)
        self._run(Event.AFTER_LOSS)
        st.loss.backward()
        return st.loss.detach()

    def _update(self):
        self._grad_mean(wait=False)
        self._run(Event.AFTER_BACKWARD)
        self.optimizer.step()

    def capture(self, batch, warmup=3):
        """Warm up on a side stream (allocations, library init, optimizer state), then
        capture the backward graph and the update graph."""
        if self.grad_accum != 1:
            raise NotImplementedError("graph mode captures one microbatch per step; "
                                      "use train_step() for grad_accum > 1")
        # drop every reference to earlier autograd graphs (outputs / loss of eager steps):
        # their AccumulateGrad nodes are bound to the stream they ran on, and a backward on
        # the capture stream that reuses them would synchronise with it and break capture
        self.state.outputs = self.state.loss = None
        torch.cuda.synchronize()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self.train_step(batch)
        torch.cuda.current_stream().wait_stream(side)
        self.state.outputs = self.state.loss = None
        torch.cuda.synchronize()
        self.buckets.defer = True
        # gradients allocated inside the graph's pool, kept across replays (with buckets the
        # hooks copy them into the bucket views and leave .grad = view)
        self.buckets.reset()
        self._g_bwd = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g_bwd):
            self._g_loss = self._forward_backward(batch)
        # lr / decay: the fused update reads them from a device array refreshed before each
        # replay (a schedule keeps working); a foreach update has them baked in as constants
        if hasattr(self.optimizer, "enable_device_hyper"):
            self.optimizer.enable_device_hyper(batch[0].device)
        self._cap_lrs = [g["lr"] for g in self.optimizer.param_groups]
        self._g_upd = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g_upd, pool=self._g_bwd.pool()):
            self._update()
        self._live_hyper = getattr(self.optimizer, "hyper_used", False)
        torch.cuda.synchronize()

    def replay(self):
        if self._live_hyper:
            self.optimizer.refresh_hyper()
        elif [g["lr"] for g in self.optimizer.param_groups] != self._cap_lrs:
            raise RuntimeError("the captured optimizer update has its learning rates baked in "
                               "(foreach path); a changed lr needs a new capture()")
        self._g_bwd.replay()
        if self.buckets.enabled:
            self.buckets.allreduce_now()
        self._g_upd.replay()
        self.state.timestamp_batch += 1
        self._run(Event.BATCH_END)
        return self._g_loss
