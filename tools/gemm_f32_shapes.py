"""fp32 NT GEMM (the parity-mode prefill Linears on the fp32 MFMA) at the
batch-1 plugin's shapes (and two 8192-row ones), µs per launch and TF/s.
    python tools/gemm_f32_shapes.py            (SMER_HIP_LIB selects a variant build)"""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(1050, 1536, 512), (1050, 512, 512), (1050, 2048, 512), (1050, 512, 2048), (1050, 1024, 512),
          (8192, 1536, 512), (8192, 512, 2048)]


def one():
    import torch
    from smer_music_generation_amd import ops
    res = {}
    for M, N, K in SHAPES:
        x = torch.randn(M, K, device="cuda")
        w = torch.randn(N, K, device="cuda")
        b = torch.randn(N, device="cuda")
        for _ in range(3):
            ops.linear(x, w, b)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ops.linear(x, w, b)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 20
        res["%dx%dx%d" % (M, N, K)] = [round(us, 1), round(2 * M * N * K / us / 1e6, 1)]
    print(json.dumps(res))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "one":
    one()
elif __name__ == "__main__":
    out = subprocess.run([sys.executable, os.path.abspath(__file__), "one"], capture_output=True, text=True,
                         timeout=300)
    print(out.stdout.strip().splitlines()[-1] if out.returncode == 0 else out.stderr[-2000:], flush=True)
