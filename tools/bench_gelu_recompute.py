import sys, torch
sys.path.insert(0, '.')
from tools.bench_skinny import timeit
from hvamd import _lib, ops
P, st = _lib.ptr, _lib.stream
M, C = 802816, 96
x = torch.randn(M, C, device="cuda").bfloat16()
w1 = (torch.randn(4*C, C, device="cuda")/C**0.5).bfloat16(); b1 = torch.randn(4*C, device="cuda")
h = torch.empty(M, 4*C, device="cuda", dtype=torch.bfloat16); y1 = torch.empty_like(h)
w2 = (torch.randn(C, 4*C, device="cuda")/(4*C)**0.5).bfloat16()
y = torch.empty(M, C, device="cuda", dtype=torch.bfloat16)
g = torch.randn(M, C, device="cuda").bfloat16()
print("fc1+gelu (h,y)", timeit(lambda: _lib.call("hvk_linear_gelu_fwd", P(x), P(w1), P(b1), P(h), P(y1), M, C, 4*C, st())))
print("fc1 h only    ", timeit(lambda: _lib.call("hvk_linear_fwd", P(x), P(w1), P(b1), P(h), M, C, 4*C, st())))
print("fc2 on y      ", timeit(lambda: _lib.call("hvk_linear_fwd", P(y1), P(w2), None, P(y), M, 4*C, C, st())))
print("fc2 gelu(h)   ", timeit(lambda: _lib.call("hvk_linear_gelu_in_fwd", P(h), P(w2), None, P(y), M, 4*C, C, st())))
print("dW2 on y      ", timeit(lambda: ops.weight_grad(g, y1, True)))
print("dW2 gelu(h)   ", timeit(lambda: ops.weight_grad(g, h, True, gelu_x=True)))
