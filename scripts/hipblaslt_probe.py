"""Reference point for the GEMM core: plain bf16 torch.matmul (hipBLASLt) rates at the
model's GEMM shapes, so the bf16x3 kernels' issue rate (3 MFMAs per product) can be set
beside what the vendor library reaches on one bf16 pass.  Not part of any product path."""
import json
import torch

dev = "cuda:0"
shapes = {  # name: (M, K, N)
    "h_fc1": (64000, 768, 3072), "h_fc2": (64000, 3072, 768), "h_qkv": (64000, 768, 2304),
    "h_cnn.c1 (im2col)": (344000, 1536, 512), "ecapa CxC": (127488, 1024, 1024),
    "ecapa conv_cat": (127488, 3072, 1536), "square 8192": (8192, 8192, 8192),
}
out = {}
for name, (M, K, N) in shapes.items():
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    e0.record()
    for _ in range(n):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    out[name] = {"M": M, "K": K, "N": N, "ms": round(ms, 4), "tflops": round(2.0 * M * K * N / ms / 1e9, 1)}
    print(name, out[name], flush=True)
    del a, b, c
print(json.dumps(out))
