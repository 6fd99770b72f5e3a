"""Library reference for the long-prompt GEMM: torch.matmul (hipBLASLt on ROCm) in fp16 with
fp32 accumulation at the codegen-16B prompt shapes, random data, Y[N][M] = X[N][K] W[M][K]^T."""
import torch


def main(reps=20):
    for M, K, N in [(6144, 6144, 2048), (24576, 6144, 2048), (6144, 24576, 2048)]:
        w = (torch.randn(M, K, device="cuda") * 0.05).half()
        x = (torch.randn(N, K, device="cuda") * 0.5).half()
        for _ in range(3):
            y = x @ w.t()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            y = x @ w.t()
        e1.record()
        torch.cuda.synchronize()
        us = 1e3 * e0.elapsed_time(e1) / reps
        print(f"torch fp16 M={M} K={K} N={N}: {us:.1f} us  {2.0 * M * K * N / us / 1e6:.0f} TFLOP/s")


if __name__ == "__main__":
    main()
