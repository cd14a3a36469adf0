"""A forward (persistent, plain epilogue) and a weight-gradient GEMM of the same shape (ffn-in:
T = 262144, 3072 x 768), five launches each: the target of the PMC passes in tools/gpu/pmc_wgrad.sh."""
import torch

from distributed_pipeline_amd.ops._ext import get_ext


def main():
    ext = get_ext(required=True)
    torch.manual_seed(0)
    T, N, K = 262144, 3072, 768
    x = torch.randn(T, K, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") * 0.03).bfloat16()
    dy = torch.randn(T, N, device="cuda").bfloat16()
    dW = torch.zeros(N, K, device="cuda")
    for _ in range(5):
        ext.gemm_nt(x, W, None, 0)
        ext.gemm_wgrad(dy, x, dW, None)
        ext.gemm_nn(dy, W)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
