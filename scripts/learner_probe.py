import torch, time
x = torch.randn(4096, 1088, device="cuda")
w = torch.randn(128, 1088, device="cuda") * 0.03
b = torch.randn(128, device="cuda")
def t(fn, n=50):
    for _ in range(5): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1000
r1 = torch.relu(torch.nn.functional.linear(x, w, b))
r2 = torch._addmm_activation(b, x, w.t())
print("maxdiff", (r1 - r2).abs().max().item())
print("linear+relu us", t(lambda: torch.relu(torch.nn.functional.linear(x, w, b))))
print("addmm_act us", t(lambda: torch._addmm_activation(b, x, w.t())))
print("linear us", t(lambda: torch.nn.functional.linear(x, w, b)))
g = torch.randn(4096, 2, device="cuda"); h = torch.randn(4096, 128, device="cuda")
print("skinny dW us", t(lambda: g.t() @ h))
print("skinny dW (h^T g) us", t(lambda: h.t() @ g))
print(torch.backends.cuda.preferred_blas_library())
