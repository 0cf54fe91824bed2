"""Probe: library (hipBLASLt via torch.matmul) bf16 GEMM rate on the ECAPA GEMM
shapes, to price a library-GEMM split-precision path against conv_gemm_x3."""
import time, torch
dev = "cuda"
def rate(M, N, K, dt=torch.bfloat16, it=20):
    a = torch.randn(M, K, device=dev, dtype=dt); b = torch.randn(K, N, device=dev, dtype=dt)
    for _ in range(3): c = a @ b
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(it): c = a @ b
    torch.cuda.synchronize(); dt_ = (time.perf_counter() - t) / it
    return dt_ * 1e3, 2 * M * N * K / dt_ / 1e12
for (M, N, K) in [(127488, 1024, 1024), (127488, 1024, 2048), (127488, 1024, 3072),
                  (127488, 1536, 3072), (127488, 1536, 9216), (16000, 3072, 768), (16000, 768, 3072)]:
    for dt in (torch.bfloat16, torch.float32):
        ms, tf = rate(M, N, K, dt)
        print(f"M={M} N={N} K={K} {dt}: {ms:.3f} ms {tf:.1f} TFLOP/s", flush=True)
