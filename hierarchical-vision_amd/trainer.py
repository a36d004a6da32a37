"""One training step with the event order composer.Trainer uses for the hot path
(SURVEY.md §3.2): forward -> BEFORE_LOSS -> loss -> AFTER_LOSS -> backward (with
bucketed RCCL all-reduce overlapped) -> AFTER_BACKWARD (clipping) -> optimizer
step -> BATCH_END (EMA).  bf16 autocast on the GPU; no host synchronisation
inside the step."""
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
