"""Library-GEMM timings for the C3 shapes (diagnostic): fp32 mm, bf16 mm (bf16 out), bf16 mm with
fp32 out (aten::mm.dtype), and the casts, for x [M, K] @ W^T [K, N] and dW = dy^T x."""
import torch

dev = torch.device("cuda:0")
M, N = 40960, 128


def t(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for K in (1025, 128):
    x = torch.randn(M, K, device=dev)
    W = torch.randn(N, K, device=dev)
    dy = torch.randn(M, N, device=dev)
    xb, Wb, dyb = x.bfloat16(), W.bfloat16(), dy.bfloat16()
    print(f"K={K}")
    print(f"  fwd fp32 mm            {t(lambda: torch.mm(x, W.t())):8.1f} us")
    print(f"  fwd bf16 mm (bf16 out) {t(lambda: torch.mm(xb, Wb.t())):8.1f} us")
    print(f"  fwd bf16 mm (f32 out)  {t(lambda: torch.mm(xb, Wb.t(), out_dtype=torch.float32)):8.1f} us")
    print(f"  fwd bf16 F.linear      {t(lambda: torch.nn.functional.linear(xb, Wb)):8.1f} us")
    print(f"  dW fp32                {t(lambda: torch.mm(dy.t(), x)):8.1f} us")
    print(f"  dW bf16 (f32 out)      {t(lambda: torch.mm(dyb.t(), xb, out_dtype=torch.float32)):8.1f} us")
    print(f"  dW bf16 (bf16 out)     {t(lambda: torch.mm(dyb.t(), xb)):8.1f} us")
    print(f"  cast x -> bf16         {t(lambda: x.bfloat16()):8.1f} us")

print("split-K dW = sum_s dy_s^T x_s (bmm over S row chunks, then a fixed-order sum)")
for K in (1025, 128):
    x = torch.randn(M, K, device=dev)
    dy = torch.randn(M, N, device=dev)
    for S in (8, 16, 32, 64):
        m = M // S
        xs, ds = x.view(S, m, K), dy.view(S, m, N)
        xb, db = xs.bfloat16(), ds.bfloat16()
        f32 = t(lambda: torch.bmm(ds.transpose(1, 2), xs).sum(0))
        b16 = t(lambda: torch.bmm(db.transpose(1, 2), xb, out_dtype=torch.float32).sum(0))
        print(f"  K={K} S={S:3d}: fp32 {f32:8.1f} us   bf16->f32 {b16:8.1f} us")
