"""Optimizer construction (optim.py): parameter groups with the reference's
no-decay rule and multi-tensor (foreach) update kernels.

Quirk kept from the reference: build_optimizer is handed the Composer wrapper,
which has no `no_weight_decay`, so the skip set is always empty and 3-D
`logit_scale` is decayed (optim.py:9-14, 53)."""
import torch

from .options import OPTIONS


def set_weight_decay(model, skip_list=()):
    """1-D params and `.bias` -> no decay (optim.py:48-58)."""
    has_decay, no_decay = [], []
    for name, param in model.named_parameters():
        if not param.requires_grad:
            continue
        if len(param.shape) == 1 or name.endswith(".bias") or (name in skip_list):
            no_decay.append(param)
        else:
            has_decay.append(param)
    return [{"params": has_decay}, {"params": no_decay, "weight_decay": 0.0}]


class DecoupledSGDW(torch.optim.Optimizer):
    """SGD + momentum with weight decay decoupled from the gradient and scaled by
    lr / initial_lr (composer.optim.DecoupledSGDW semantics).

    On the GPU one step is libhvk's fused hvk_sgdw_step (include/hvk.h), which also takes the
    hand-overs of the step's other per-parameter passes so none of them reads the 141 MB of
    gradients or weights again: ``pending_grad_scale`` (1/world: the DDP buckets hold gradient
    SUMS, ddp.py), ``pending_clip`` (GradientClipping's norm threshold) and ``pending_ema``
    (the EMA algorithm's averaged copies on the batches it updates them).  Elsewhere the same
    step runs as foreach passes."""

    def __init__(self, params, lr, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False):
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov, initial_lr=lr)
        super().__init__(params, defaults)

        self.pending_clip = None  # global-norm threshold handed over by GradientClipping
        self.pending_grad_scale = 1.0  # gradient multiplier handed over by the trainer (DDP mean)
        self.pending_ema = None  # ([(id(param), ema tensor)], smoothing) from the EMA algorithm
        self.device_hyper = False  # graph mode: lr / decay read from a device array at run time
        self._hyper = None
        self._fused = None

    def supports_fused_clip(self):
        return True

    def supports_grad_scale(self):
        return True

    def supports_fused_ema(self, params):
        """The fused step can apply an EMA over exactly these parameters when every one of them
        is in a param group (the trainer asks before handing the EMA over)."""
        mine = {id(p) for g in self.param_groups for p in g["params"]}
        return self._fused_eligible() and mine == {id(p) for p in params}

    def _fused_eligible(self):
        if not OPTIONS.fused_optim:  # A/B runs: the foreach path
            return False
        gs = self.param_groups
        if not gs or any(g["nesterov"] != gs[0]["nesterov"] or g["momentum"] != gs[0]["momentum"]
                         or g["dampening"] != gs[0]["dampening"] for g in gs):
            return False
        for g in gs:
            for p in g["params"]:
                if p.grad is None:
                    continue
                if not (p.is_cuda and p.dtype == torch.float32 and p.grad.dtype == torch.float32
                        and p.is_contiguous() and p.grad.is_contiguous()):
                    return False
        return gs[0]["momentum"] != 0 and len(gs) <= 4

    def _hyper_values(self):
        gs = self.param_groups
        lr = [float(g["lr"]) for g in gs] + [0.0] * (4 - len(gs))
        decay = [1.0 - g["weight_decay"] * g["lr"] / g["initial_lr"] if g["weight_decay"] else 1.0
                 for g in gs] + [1.0] * (4 - len(gs))
        return lr, decay

    def enable_device_hyper(self, device):
        """Graph mode (trainer.capture): the fused update reads lr / decay from a device array
        instead of kernel arguments, so a schedule still applies to captured replays."""
        lr, decay = self._hyper_values()
        self._hyper = torch.tensor(lr + decay, dtype=torch.float32, device=device)
        self._hyper_ring = [(torch.empty(8, dtype=torch.float32).pin_memory(), None) for _ in range(4)]
        self._hyper_slot = 0
        self.device_hyper = True
        self.hyper_used = False

    def refresh_hyper(self):
        """Copy the current lr / decay of every group into that device array, stream-ordered
        before the next replay (a ring of pinned staging buffers: no host sync per step)."""
        if self._hyper is None:
            return
        lr, decay = self._hyper_values()
        host, ev = self._hyper_ring[self._hyper_slot]
        if ev is not None:
            ev.synchronize()  # that slot's previous copy (4 steps ago) has been consumed
        host.copy_(torch.tensor(lr + decay, dtype=torch.float32))
        self._hyper.copy_(host, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._hyper_ring[self._hyper_slot] = (host, ev)
        self._hyper_slot = (self._hyper_slot + 1) % len(self._hyper_ring)

    def _fused_step(self):
        """Mean + clip + update (+ EMA) of every tensor in a handful of libhvk launches
        (hvk_sgdw_step); False (nothing done) when only some momentum buffers exist yet."""
        import ctypes
        from . import _lib
        ps, grp = [], []
        for gi, g in enumerate(self.param_groups):
            for p in g["params"]:
                if p.grad is not None:
                    ps.append(p)
                    grp.append(gi)
        if not ps:
            return True
        fresh = ["momentum_buffer" not in self.state[p] for p in ps]
        if any(fresh) and not all(fresh):
            return False
        first = all(fresh)
        if first:  # torch SGD semantics: the first step's buffer is the (clipped) gradient
            for p in ps:
                self.state[p]["momentum_buffer"] = torch.empty_like(p)
        n = len(ps)
        P = ctypes.c_void_p * n
        numel = (ctypes.c_longlong * n)(*[p.numel() for p in ps])
        arrs = [P(*[p.data_ptr() for p in ps]), P(*[p.grad.data_ptr() for p in ps]),
                P(*[self.state[p]["momentum_buffer"].data_ptr() for p in ps])]
        ema_arr, ema_a = None, 0.0
        if self.pending_ema is not None:
            emas, ema_a = self.pending_ema
            by_id = dict(emas)
            ema_arr = P(*[by_id[id(p)].data_ptr() for p in ps])
        gs = self.param_groups
        lr_v, decay_v = self._hyper_values()
        lr = (ctypes.c_float * 4)(*lr_v)
        decay = (ctypes.c_float * 4)(*decay_v)
        hyper = None
        # the device array only inside a capture (replay() refreshes it); an eager step takes
        # the current lr / decay as arguments, so a schedule change is never missed
        if self.device_hyper and self._hyper is not None and torch.cuda.is_current_stream_capturing():
            hyper = _lib.ptr(self._hyper)
            self.hyper_used = True
        lib = _lib.load()
        nb = lib.hvk_sgdw_workspace_bytes(n, ctypes.cast(numel, ctypes.c_void_p))
        if self._fused is None or self._fused.numel() * 4 < nb:
            self._fused = torch.empty(nb // 4, device=ps[0].device, dtype=torch.float32)
        clip = float(self.pending_clip) if self.pending_clip is not None else 0.0
        g0 = gs[0]
        self._keep = (arrs, ema_arr, numel)  # ctypes tables outlive the call
        _lib.call("hvk_sgdw_step", n, *[ctypes.cast(a, ctypes.c_void_p) for a in arrs],
                  ctypes.cast(ema_arr, ctypes.c_void_p) if ema_arr is not None else None,
                  ctypes.cast(numel, ctypes.c_void_p), ctypes.cast((ctypes.c_int * n)(*grp), ctypes.c_void_p),
                  ctypes.cast(lr, ctypes.c_void_p), ctypes.cast(decay, ctypes.c_void_p), len(gs), hyper,
                  float(self.pending_grad_scale), clip, float(g0["momentum"]), float(g0["dampening"]),
                  int(bool(g0["nesterov"])), int(first), float(ema_a), _lib.ptr(self._fused), nb,
                  _lib.stream())
        # the kernel wrote the weights through raw pointers: bump their version counters so
        # version-keyed caches (ops._WeightCopies) see the update
        torch.autograd.graph.increment_version(ps)
        return True

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        try:
            if self._fused_eligible() and self._fused_step():
                return loss
            self._foreach_step()
        finally:
            self.pending_clip = None
            self.pending_grad_scale = 1.0
            self.pending_ema = None
        return loss

    def _foreach_step(self):
        params = [p for g in self.param_groups for p in g["params"] if p.grad is not None]
        if self.pending_grad_scale != 1.0 and params:
            torch._foreach_mul_([p.grad for p in params], float(self.pending_grad_scale))
        if self.pending_clip is not None:  # unfused: clip now, as GradientClipping would
            torch.nn.utils.clip_grad_norm_(params, self.pending_clip, foreach=True)
        for g in self.param_groups:
            ps = [p for p in g["params"] if p.grad is not None]
            if not ps:
                continue
            grads = [p.grad for p in ps]
            lr, mom, wd = g["lr"], g["momentum"], g["weight_decay"]
            if mom != 0:
                fresh = [p for p in ps if "momentum_buffer" not in self.state[p]]
                seen = set(map(id, fresh))
                old = [p for p in ps if id(p) not in seen]
                for p in fresh:  # first step: buffer = grad (torch.optim.SGD semantics)
                    self.state[p]["momentum_buffer"] = p.grad.detach().clone()
                if old:
                    bl = [self.state[p]["momentum_buffer"] for p in old]
                    torch._foreach_mul_(bl, mom)
                    torch._foreach_add_(bl, [p.grad for p in old], alpha=1 - g["dampening"])
                bl = [self.state[p]["momentum_buffer"] for p in ps]
                grads = torch._foreach_add(grads, bl, alpha=mom) if g["nesterov"] else bl
            if wd != 0:
                torch._foreach_mul_(ps, 1 - wd * lr / g["initial_lr"])
            torch._foreach_add_(ps, grads, alpha=-lr)
        if self.pending_ema is not None:
            emas, a = self.pending_ema
            by_id = dict(emas)
            ps = [p for p in params if id(p) in by_id]
            es = [by_id[id(p)] for p in ps]
            torch._foreach_mul_(es, a)
            torch._foreach_add_(es, ps, alpha=1 - a)


def build_optimizer(config, model):
    skip = model.no_weight_decay() if hasattr(model, "no_weight_decay") else {}
    parameters = set_weight_decay(model, skip)
    name = config.optim.name.lower()
    o = config.optim
    if name == "sgd":
        return torch.optim.SGD(parameters, momentum=o.momentum, nesterov=True, lr=o.lr,
                               weight_decay=o.weight_decay, foreach=True)
    if name == "adamw":
        return torch.optim.AdamW(parameters, lr=o.lr, weight_decay=o.weight_decay, foreach=True)
    if name == "decoupledadamw":
        return torch.optim.AdamW(parameters, lr=o.lr, weight_decay=o.weight_decay / o.lr,
                                 foreach=True)
    if name == "decoupledsgdw":
        return DecoupledSGDW(parameters, lr=o.lr, momentum=o.momentum, weight_decay=o.weight_decay)
    raise ValueError(name)
