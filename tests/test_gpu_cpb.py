"""Fused CPB table + logit scale (hvk_cpb_fwd/bwd) vs torch f32 autograd of the same
modules (swinv2.py:141-145, 230-246)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("win,pw,nh", [(7, 0, 3), (8, 8, 24), (24, 12, 32), (12, 0, 4)])
def test_cpb_table_and_grads(win, pw, nh):
    from hvamd import ops, swinv2
    torch.manual_seed(win * 100 + nh)
    coords = swinv2.relative_coords_table((win, win), (pw, pw)).reshape(-1, 2).cuda().float()
    mlp = torch.nn.Sequential(torch.nn.Linear(2, 512), torch.nn.ReLU(),
                              torch.nn.Linear(512, nh, bias=False)).cuda()
    logit = torch.log(10 * torch.ones(nh, 1, 1, device="cuda")) + 0.3 * torch.randn(nh, 1, 1, device="cuda")
    logit[0] = 6.0  # above the clamp: zero gradient
    logit.requires_grad_(True)
    cmax = float(torch.log(torch.tensor(100.0)))
    table, scale = ops.cpb_table(coords, mlp[0].weight, mlp[0].bias, mlp[2].weight, logit, cmax)
    gt = torch.randn_like(table)
    gs = torch.randn_like(scale)
    (table * gt).sum().add_((scale * gs).sum()).backward()
    mine = [table.detach(), scale.detach(), mlp[0].weight.grad.clone(), mlp[0].bias.grad.clone(),
            mlp[2].weight.grad.clone(), logit.grad.clone()]
    for p in list(mlp.parameters()) + [logit]:
        p.grad = None
    rt = (16 * torch.sigmoid(mlp(coords))).t()
    rs = torch.clamp(logit, max=cmax).exp().reshape(-1)
    (rt * gt).sum().add_((rs * gs).sum()).backward()
    ref = [rt.detach(), rs.detach(), mlp[0].weight.grad, mlp[0].bias.grad, mlp[2].weight.grad,
           logit.grad]
    for name, a, b in zip(["table", "scale", "dw1", "db1", "dw2", "dlogit"], mine, ref):
        rel = ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
        assert rel < 1e-4, (name, rel)
    assert mine[5][0].abs().item() == 0.0
