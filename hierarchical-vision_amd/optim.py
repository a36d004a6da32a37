"""Optimizer construction (optim.py): parameter groups with the reference's
no-decay rule and multi-tensor (foreach) update kernels.

Quirk kept from the reference: build_optimizer is handed the Composer wrapper,
which has no `no_weight_decay`, so the skip set is always empty and 3-D
`logit_scale` is decayed (optim.py:9-14, 53)."""
import os

import torch


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
    lr / initial_lr (composer.optim.DecoupledSGDW semantics), foreach kernels."""

    def __init__(self, params, lr, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False):
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov, initial_lr=lr)
        super().__init__(params, defaults)

        self.pending_clip = None  # global-norm threshold handed over by GradientClipping
        self._fused = None

    def supports_fused_clip(self):
        return True

    def _fused_eligible(self):
        if os.environ.get("HVK_FUSED_OPTIM", "1") == "0":  # A/B runs: the foreach path
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

    def _fused_step(self):
        """Clip + update of every tensor in a handful of libhvk launches (hvk_sgdw_step);
        False (nothing done) when only some momentum buffers exist yet."""
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
        arrs = (P(*[p.data_ptr() for p in ps]), P(*[p.grad.data_ptr() for p in ps]),
                P(*[self.state[p]["momentum_buffer"].data_ptr() for p in ps]), numel,
                (ctypes.c_int * n)(*grp))
        gs = self.param_groups
        lr = (ctypes.c_float * len(gs))(*[g["lr"] for g in gs])
        decay = (ctypes.c_float * len(gs))(
            *[1.0 - g["weight_decay"] * g["lr"] / g["initial_lr"] if g["weight_decay"] else 1.0
              for g in gs])
        lib = _lib.load()
        nb = lib.hvk_sgdw_workspace_bytes(n, ctypes.cast(numel, ctypes.c_void_p))
        if self._fused is None or self._fused.numel() * 4 < nb:
            self._fused = torch.empty(nb // 4, device=ps[0].device, dtype=torch.float32)
        clip = float(self.pending_clip) if self.pending_clip is not None else 0.0
        g0 = gs[0]
        _lib.call("hvk_sgdw_step", n, *[ctypes.cast(a, ctypes.c_void_p) for a in arrs],
                  ctypes.cast(lr, ctypes.c_void_p), ctypes.cast(decay, ctypes.c_void_p), len(gs),
                  clip, float(g0["momentum"]), float(g0["dampening"]), int(bool(g0["nesterov"])),
                  int(first), _lib.ptr(self._fused), nb, _lib.stream())
        return True

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        if self._fused_eligible() and self._fused_step():
            self.pending_clip = None
            return loss
        if self.pending_clip is not None:  # unfused: clip now, as GradientClipping would
            params = [p for g in self.param_groups for p in g["params"] if p.grad is not None]
            torch.nn.utils.clip_grad_norm_(params, self.pending_clip, foreach=True)
            self.pending_clip = None
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
        return loss


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
