"""Times the C2 training step's GEMM shapes (bf16, N = 8192 tokens) under hipBLASLt and rocBLAS, including the
weight-gradient products in both operand orders."""
import torch

N = 8192
SHAPES = [(768, 256), (256, 256), (1024, 256), (256, 1024), (1232, 256)]


def t(fn, it=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


for lib in ("cublaslt", "cublas"):
    try:
        torch.backends.cuda.preferred_blas_library(lib)
    except Exception as ex:  # noqa: BLE001
        print(lib, "unavailable", ex)
        continue
    for out, inn in SHAPES:
        x = torch.randn(N, inn, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(out, inn, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(N, out, device="cuda", dtype=torch.bfloat16)
        fl = 2 * N * out * inn
        r = {
            "fwd": t(lambda: torch.nn.functional.linear(x, w)),
            "dX": t(lambda: dy @ w),
            "dW=dyT@x": t(lambda: dy.t() @ x),
            "dWT=xT@dy": t(lambda: x.t() @ dy),
        }
        try:
            r["dW f32out"] = t(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
        except Exception:  # noqa: BLE001
            pass
        print(lib, (out, inn), "  ".join(f"{k} {v:6.1f}us ({fl / v / 1e6:5.0f}TF)" for k, v in r.items()), flush=True)

# the HIP projection GEMM (csrc/gemm.hip) on the same shapes
import os, sys  # noqa: E401,E402
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eventstreamgpt_amd.fused import linear_dw, linear_dx, linear_fwd  # noqa: E402

for out, inn in SHAPES:
    x = torch.randn(N, inn, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(out, inn, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(N, out, device="cuda", dtype=torch.bfloat16)
    fl = 2 * N * out * inn
    r = {"fwd": t(lambda: linear_fwd(x, w)), "dX": t(lambda: linear_dx(dy, w)), "dW f32": t(lambda: linear_dw(dy, x))}
    print("hip", (out, inn), "  ".join(f"{k} {v:6.1f}us ({fl / v / 1e6:5.0f}TF)" for k, v in r.items()), flush=True)
