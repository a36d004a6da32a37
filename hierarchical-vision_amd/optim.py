"""Optimizer construction (optim.py): parameter groups with the reference's
no-decay rule and multi-tensor (foreach) update kernels.

Quirk kept from the reference: build_optimizer is handed the Composer wrapper,
which has no `no_weight_decay`, so the skip set is always empty and 3-D
`logit_scale` is decayed (optim.py:9-14, 53)."""
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

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
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
