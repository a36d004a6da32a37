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
import torch

from .algorithmic import Event, State
from .ddp import GradientBuckets


class Trainer:
    def __init__(self, model, optimizer, algorithms=(), bucket_mb=64.0, dtype=torch.bfloat16,
                 device_transforms=None):
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
        self._run(Event.INIT)

    def _run(self, event):
        for a in self.algorithms:
            if a.match(event, self.state):
                a.apply(event, self.state, None)

    def train_step(self, batch):
        st = self.state
        if self.device_transforms is not None:
            batch = self.device_transforms(batch)
        st.batch = batch
        self.model.train()
        dev_type = batch[0].device.type
        with torch.autocast(device_type=dev_type, dtype=self.dtype, enabled=dev_type == "cuda"):
            st.outputs = self.model(st.batch)
        self._run(Event.BEFORE_LOSS)
        st.loss = self.model.loss(st.outputs, st.batch)
        self._run(Event.AFTER_LOSS)
        st.loss.backward()
        self._grad_mean()
        self._run(Event.AFTER_BACKWARD)
        self.optimizer.step()
        self.buckets.reset()
        st.timestamp_batch += 1
        self._run(Event.BATCH_END)
        return st.loss.detach()

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
