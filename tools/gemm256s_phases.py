"""Phase split of the staggered 256x256 GEMM from in-kernel s_memtime stamps
(smer_gemm_debug_stamps): per tile, the prologue (first k-steps' DMA until
the k-loop starts), the k-loop, and the epilogue, in core cycles, for the
loader (waves 4-7) and storer (waves 0-3) halves, median over workgroups.

    python tools/gemm256s_phases.py
"""
import ctypes
import os
import sys

os.environ["SMER_GEMM256S"] = "1"  # the kernel is opt-in

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from smer_music_generation_amd import _lib, ops  # noqa: E402

SHAPES = [("fwd ffn1 brd", 32768, 2048, 512, True, "brd"), ("fwd qkv b", 32768, 1536, 512, True, "b"),
          ("fwd ffn2 bR", 32768, 512, 2048, True, "bR"), ("dgrad ffn1 R", 32768, 512, 2048, False, "R"),
          ("dgrad ffn2 g", 32768, 2048, 512, False, "g")]


def main():
    lib = _lib.load()
    dev = "cuda"
    bf = torch.bfloat16
    buf = torch.zeros(256 * 64 + 64, dtype=torch.int64, device=dev)
    for name, M, N, K, bk, epi in SHAPES:
        A = torch.randn(M, K, device=dev).to(bf)
        W = (torch.randn(N, K, device=dev) * 0.05).to(bf)
        Wm = W if bk else W.t().contiguous()
        X = torch.randn(M, N, device=dev).to(bf)
        C = torch.empty(M, N, device=dev, dtype=bf)
        kw = {}
        if "b" in epi:
            kw["bias"] = torch.randn(N, device=dev)
        if "r" in epi:
            kw["relu"] = True
        if "d" in epi:
            kw["drop_p"], kw["seed"] = 0.1, 3
        if "R" in epi:
            kw["residual"] = X
        if "g" in epi:
            kw["gate"] = X
        for _ in range(3):
            ops.gemm(A, Wm, M=M, N=N, K=K, b_kcontig=bk, out=C, **kw)
        torch.cuda.synchronize()
        buf.zero_()
        lib.smer_gemm_debug_stamps(ctypes.c_void_p(buf.data_ptr()), buf.numel() * buf.element_size())
        ops.gemm(A, Wm, M=M, N=N, K=K, b_kcontig=bk, out=C, **kw)
        torch.cuda.synchronize()
        lib.smer_gemm_debug_stamps(ctypes.c_void_p(0), 0)
        st = buf[:256 * 64].view(256, 8, 8).cpu().numpy().astype(np.float64)
        nk = K // 32
        for tile in (0, 1):
            s = st[:, :, 4 * tile:4 * tile + 4]
            ok = s[:, :, 0] > 0
            if not ok.any():
                continue
            pro = s[:, :, 1] - s[:, :, 0]
            loop = s[:, :, 2] - s[:, :, 1]
            epi_ = s[:, :, 3] - s[:, :, 2]
            row = []
            for grp, sl in (("storers", slice(0, 4)), ("loaders", slice(4, 8))):
                m = ok[:, sl]
                row.append("%s prologue %6.0f loop %7.0f (%5.0f/k-step) epilogue %6.0f" % (
                    grp, np.median(pro[:, sl][m]), np.median(loop[:, sl][m]), np.median(loop[:, sl][m]) / nk,
                    np.median(epi_[:, sl][m])))
            print("%-14s tile %d: %s" % (name, tile, " | ".join(row)), flush=True)
        # tile-to-tile gap (epilogue end of tile 0 -> start of tile 1)
        ok = (st[:, :, 4] > 0)
        if ok.any():
            print("%-14s gap tile0 end -> tile1 start %6.0f cycles" % (name, np.median((st[:, :, 4] - st[:, :, 3])[ok])))
        del A, W, Wm, X, C
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
