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
    def __init__(self, model, optimizer, algorithms=(), bucket_mb=64.0, dtype=torch.bfloat16):
        self.model = model
        self.optimizer = optimizer
        self.algorithms = list(algorithms)
        self.dtype = dtype
        self.state = State(model, optimizer)
        self.buckets = GradientBuckets(model, bucket_mb=bucket_mb)
        self._run(Event.INIT)

    def _run(self, event):
        for a in self.algorithms:
            if a.match(event, self.state):
                a.apply(event, self.state, None)

    def train_step(self, batch):
        st = self.state
        st.batch = batch
        self.model.train()
        dev_type = batch[0].device.type
        with torch.autocast(device_type=dev_type, dtype=self.dtype, enabled=dev_type == "cuda"):
            st.outputs = self.model(st.batch)
        self._run(Event.BEFORE_LOSS)
        st.loss = self.model.loss(st.outputs, st.batch)
        self._run(Event.AFTER_LOSS)
        st.loss.backward()
        self.buckets.synchronize()
        self._run(Event.AFTER_BACKWARD)
        self.optimizer.step()
        self.buckets.reset()
        st.timestamp_batch += 1
        self._run(Event.BATCH_END)
        return st.loss.detach()

    # ---------------------------------------------------------------- graph mode
    def _forward_backward(self, batch):
        st = self.state
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
        if self.buckets.enabled:
            self.buckets.scale_()
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
        if not self.buckets.enabled:
            for p in self.model.parameters():
                p.grad = None  # allocated inside the graph's pool, kept across replays
        self._g_bwd = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g_bwd):
            self._g_loss = self._forward_backward(batch)
        self._g_upd = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g_upd, pool=self._g_bwd.pool()):
            self._update()
        torch.cuda.synchronize()

    def replay(self):
        self._g_bwd.replay()
        if self.buckets.enabled:
            self.buckets.allreduce_now()
        self._g_upd.replay()
        self.state.timestamp_batch += 1
        self._run(Event.BATCH_END)
        return self._g_loss
