"""Headline benchmark: SMER train tokens/s (+ infill tokens/s) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-infill] [--no-cpu]

Workload (BASELINE.json configs[1] / SURVEY.md §8d C2): 6-layer encoder +
6-layer decoder, d_model 512, 8 heads, FF 2048, V 309, per GPU B=32 source
sequences of S=1024 SMER tokens and T=256 decoder tokens (synthetic SMER
grammar, seeded), bf16 MFMA compute with fp32 master weights, dropout 0.1
as the reference trains (train.py:257-259), the full step timed: forward,
fused weighted CE, backward, RCCL gradient all-reduce (N>1), Adam.
One step = one pass over one batch.  value = N*B*(S+T)*K / max-rank time.

Infill (second block, replicas only): batched greedy KV-cached decode of
32 requests per GPU on the same model with S~1024 sources.

Multi-GPU: launched by torch.distributed.run, one rank per GPU, RCCL.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CTRL = ['key', 'tensile', 'density', 'polyphony', 'occupation']
BF16_PEAK_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
FP8_PEAK_TFLOPS = 5000.0    # MI355X dense fp8 MFMA (block-scaled e4m3)
HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec


def train_flops_per_sample(L, d, F, V, S, T):
    """forward algorithmic flops per sample (attention dense)."""
    enc = L * (8 * S * d * d + 4 * S * d * F + 4 * S * S * d)
    dec = L * (12 * T * d * d + 4 * T * T * d + 4 * S * d * d + 4 * T * S * d + 4 * T * d * F)
    return enc + dec + 2 * T * d * V


def make_model(args, dev, precision="bf16"):
    from smer_music_generation_amd.model import ScoreTransformer
    torch.manual_seed(0)
    m = ScoreTransformer(309, args.d_model, args.nhead, args.layers, args.layers, args.ff, 2400,
                         args.dropout, args.dropout, precision=precision)
    for p in m.parameters():  # train.py:261-263
        if p.dim() > 1:
            torch.nn.init.xavier_normal_(p)
    return m.to(dev)


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def timed_steps(step, steps, warmup, dev, world):
    """The bench contract's timed region: W untimed warmup steps, then
    exactly K steps bracketed by barrier + device synchronize on both sides;
    returns (seconds of this rank, last step's result)."""
    out = None
    for _ in range(warmup):
        out = step()
    _sync(dev)
    if world > 1:
        dist.barrier()
    _sync(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step()
    _sync(dev)
    if world > 1:
        dist.barrier()
    return time.perf_counter() - t0, out


def max_over_ranks(x, dev, world):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def params_in_sync(model, dev, world):
    """True when every rank holds bit-identical parameters (after the
    Trainer's rank-0 broadcast): each rank's flat buffer hashed to two
    float64 sums, gathered and compared."""
    if world == 1:
        return True
    flat = model.flat_parameters().detach()
    idx = torch.arange(flat.numel(), device=flat.device, dtype=torch.float64) % 1021 + 1
    h = torch.stack([flat.double().sum(), (flat.double() * idx).sum()]).to(dev)
    allh = [torch.zeros_like(h) for _ in range(world)]
    dist.all_gather(allh, h)
    return all(torch.equal(allh[0], x) for x in allh[1:])


def bench_train(args, dev, rank, world, precision="bf16", grad_wire=None):
    from smer_music_generation_amd import ops
    from smer_music_generation_amd.synth import synth_training_batch
    from smer_music_generation_amd.train import Trainer
    from smer_music_generation_amd.vocab import WordVocab
    v = WordVocab(0, CTRL)
    m = make_model(args, dev, precision)
    tr = Trainer(m, v, lr=1e-4, grad_wire_dtype=grad_wire)
    in_sync = params_in_sync(m, dev, world)
    b = synth_training_batch(1000 + rank, v, args.batch, args.seq, args.tgt)
    bt = {k: torch.from_numpy(np.asarray(x)).to(dev) for k, x in b.items()}
    dt, loss = timed_steps(lambda: tr.step(bt), args.steps, args.warmup, dev, world)
    # The per-launch GEMM timing (HIP events around every smer_gemm call)
    # runs over a second, separate set of K steps so that the event records
    # do not slow the timed steps above.  Those steps run the weight
    # gradients on the main stream (SMER_WGRAD_OVERLAP=0): each launch's
    # duration is then its own, not stretched by a concurrent kernel.
    timer = None
    if args.roofline:
        timer = ops.KernelTimer()
        ops.GEMM_TIMER = timer
        prev = os.environ.get("SMER_WGRAD_OVERLAP")
        os.environ["SMER_WGRAD_OVERLAP"] = "0"
        try:
            ts0 = time.perf_counter()
            for _ in range(args.steps):
                tr.step(bt)
            torch.cuda.synchronize()
            t_serial = time.perf_counter() - ts0
        finally:
            ops.GEMM_TIMER = None
            if prev is None:
                del os.environ["SMER_WGRAD_OVERLAP"]
            else:
                os.environ["SMER_WGRAD_OVERLAP"] = prev
    dt = max_over_ranks(dt, dev, world)
    tokens = world * args.batch * (args.seq + args.tgt) * args.steps
    flops_sample = train_flops_per_sample(args.layers, args.d_model, args.ff, 309, args.seq, args.tgt)
    step_flops = 3.0 * flops_sample * args.batch  # per GPU: fwd + 2x bwd
    res = {"tokens_per_s": tokens / dt, "ms_per_step": 1000 * dt / args.steps,
           "tgt_tokens_per_s": world * args.batch * args.tgt * args.steps / dt,
           "loss": float(loss.item()), "params_in_sync_at_init": in_sync,
           "grad_allreduce_dtype": "bf16" if grad_wire == torch.bfloat16 else "fp32",
           "step_tflops_per_gpu": step_flops / (dt / args.steps) / 1e12,
           "mfma_frac_whole_step": step_flops / (dt / args.steps) / 1e12 / BF16_PEAK_TFLOPS}
    if timer is not None:
        s = timer.summary()
        achieved = s["flops"] / (s["total_ms"] / 1e3) / 1e12
        res["gemm"] = {"launches": s["launches"], "avg_us": 1000 * s["total_ms"] / max(1, s["launches"]),
                       "flops_per_launch": s["flops"] / max(1, s["launches"]),
                       "tflops": achieved,
                       # GEMM time over the wall time of the SAME (serialised) steps
                       "share_of_step": s["total_ms"] / (1000 * t_serial),
                       "timed_over": "%d extra steps after the timed ones, weight gradients "
                                     "on the main stream (no concurrent kernels)" % args.steps}
    return res


def bench_train_c4(args, dev, rank, world, precision):
    """BASELINE.json configs[3] / SURVEY §8 C4 shapes: 12 + 12 layers, d_model
    768, 12 heads, FF 2048, per-GPU B=32 sources of S=2048 and T=512 decoder
    tokens, dropout 0.1, the full train step.  precision "fp8": the QKV / FFN /
    cross-attention forward contractions on the e4m3 MFMA with delayed
    per-tensor scaling (fp8.py), everything else bf16; "bf16" for comparison."""
    import copy
    a = copy.copy(args)
    a.layers, a.d_model, a.nhead, a.seq, a.tgt = 12, 768, 12, 2048, 512
    a.steps, a.warmup, a.roofline = args.c4_steps, args.c4_warmup, False
    return bench_train(a, dev, rank, world, precision)


def _infill_requests(n, target_len=1024, seed0=0, n_infill_bars=2):
    """n synthetic 3-track songs whose MASKED source (the encoder input) holds
    at least target_len SMER tokens, each request infilling one track over
    its last-but-two n_infill_bars bars."""
    from smer_music_generation_amd.generation import _prepare
    from smer_music_generation_amd.synth import synth_events
    from smer_music_generation_amd.vocab import WordVocab
    v = WordVocab(0, CTRL)
    reqs = []
    for i in range(n):
        nb = max(8, target_len // 80)
        while True:
            ev = synth_events(seed0 + i, n_bars=nb, n_tracks=3)
            bars = list(range(nb - 2 - n_infill_bars, nb - 2))
            n_src = len(_prepare(list(ev), v, [i % 3], bars)[0])
            if n_src >= target_len:
                break
            # jump close to the target, then step bar by bar
            nb = max(nb + 1, int(nb * target_len / n_src) - 1)
        reqs.append((ev, [i % 3], bars))
    return reqs


def infill_roofline(args, st, elem=2):
    """SURVEY.md §8d infill roofline (HBM-bound): every decode step streams
    the decoder weights (L(6d^2 + 2dF) + dV bf16; the cross K/V projections
    ran at prefill) and each live request's K/V rows, L * 2d bf16 per key
    row attended (memory + prefix).  achieved = those bytes / the decode
    loop's wall time."""
    L, d, F, V = args.layers, args.d_model, args.ff, 309
    w_bytes = (L * (6 * d * d + 2 * d * F) + d * V) * elem
    if not st.get("kv_row_reads") or not st.get("step_call_s"):
        return None
    total = st["steps"] * w_bytes + st["kv_row_reads"] * L * 2 * d * elem
    gbs = total / st["step_call_s"] / 1e9
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_step": round(total / max(1, st["steps"])),
            "weight_bytes_per_step": w_bytes}


def bench_infill(args, dev, rank, precision="bf16"):
    """precision "fp32": the bit-exact decode path (greedy ids equal the
    reference's; tests/test_prod_gpu.py), same requests and method."""
    from smer_music_generation_amd.generation import generation_batch
    from smer_music_generation_amd.vocab import WordVocab
    v = WordVocab(0, CTRL)
    m = make_model(args, dev, precision).eval()
    all_controls = v.density_indices + v.occupation_indices + v.polyphony_indices + v.tensile_indices
    # the first call (other requests, sources a little longer) allocates the
    # session and captures the decode graph: timed as the cold rate; the
    # timed call then runs on that warm session, as a serving process would
    warm = _infill_requests(args.infill_batch, args.seq + 128, 900)
    torch.cuda.synchronize()
    tw = time.perf_counter()
    _, wst = generation_batch(m, warm, v, all_controls, greedy=True, return_stats=True)
    torch.cuda.synchronize()
    cold_s = time.perf_counter() - tw
    cold = wst["tokens"] / cold_s
    cold_phases = dict({k: round(wst[k], 4) for k in ("prepare_s", "prefill_s", "decode_s", "step_call_s")},
                       **{k: round(v, 4) for k, v in wst.get("decode_phases_s", {}).items()},
                       total_s=round(cold_s, 4))
    reqs = _infill_requests(args.infill_batch, args.seq, 100 * rank)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, st = generation_batch(m, reqs, v, all_controls, greedy=True, return_stats=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    src_len = float(np.mean([len(r[0]) for r in reqs]))
    return {"tokens": st["tokens"], "steps": st["steps"], "seconds": dt, "cold_tokens_per_s": cold,
            "cold_phases_s": cold_phases,
            "phases_s": dict({k: round(st[k], 4) for k in ("prepare_s", "prefill_s", "decode_s",
                                                           "step_call_s")},
                             **{k: round(v, 4) for k, v in st.get("decode_phases_s", {}).items()}),
            "tokens_per_s": st["tokens"] / dt, "requests": len(reqs), "mean_src_len": src_len,
            "ms_per_decode_step": 1000 * st["step_call_s"] / max(1, st["steps"]),
            "roofline": infill_roofline(args, st, 4 if precision == "fp32" else 2)}


def bench_infill_batch1(args, dev, rank):
    """The plugin call itself: one `generation_all` (reference signature and
    defaults: weighted sampling, batch 1, host grammar loop per token over the
    KV-cached session) on a C2-model request with an S>=1024 source."""
    from smer_music_generation_amd.generation import generation_all
    from smer_music_generation_amd.vocab import WordVocab
    v = WordVocab(0, CTRL)
    m = make_model(args, dev).eval()
    ac = v.density_indices + v.occupation_indices + v.polyphony_indices + v.tensile_indices
    (wev, wtr, wbr), = _infill_requests(1, args.seq, 8100 + rank)
    np.random.seed(1)
    # the process's first plugin call (session + graph capture): its latency
    # is the cold batch-1 figure
    torch.cuda.synchronize()
    tc = time.perf_counter()
    cst = {}
    generation_all(m, list(wev), dev, v, None, ac, wtr, wbr, stats=cst)
    torch.cuda.synchronize()
    cold_s = time.perf_counter() - tc
    reqs = _infill_requests(8, args.seq, 8000 + 100 * rank)
    from smer_music_generation_amd.generation import _prepare
    src_len = float(np.mean([len(_prepare(list(ev), v, tr, br)[0]) for ev, tr, br in reqs]))
    np.random.seed(0)
    steps = 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for ev, tr, br in reqs:  # one plugin call per request, back to back
        stats = {}
        if generation_all(m, list(ev), dev, v, None, ac, tr, br, stats=stats) is not None:
            steps += stats["steps"]
    dt = time.perf_counter() - t0
    return {"value": round(steps / dt, 1), "tokens": steps, "seconds": round(dt, 4),
            "requests": len(reqs), "mean_src_len": round(src_len, 1),
            "ms_per_token": round(1000 * dt / max(1, steps), 3),
            "cold_call_s": round(cold_s, 4), "cold_call_tokens": cst.get("steps"),
            "warm_call_s_mean": round(dt / len(reqs), 4)}


def bench_infill_c5(args, dev, rank, precision="bf16"):
    """BASELINE.json configs[4]: 64 concurrent requests,
    sources of ~4096 SMER tokens, each infilling 4 bars of one track, greedy,
    KV-cached, graph-captured decode step with the grammar on device.
    Reports tokens/s and the p50 / p90 request latency (host preparation +
    prefill + the GPU end time of the request's last decode step)."""
    from smer_music_generation_amd.generation import generation_batch
    from smer_music_generation_amd.vocab import WordVocab
    v = WordVocab(0, CTRL)
    m = make_model(args, dev, precision).eval()
    all_controls = v.density_indices + v.occupation_indices + v.polyphony_indices + v.tensile_indices
    # cold first call on other requests (session + graph capture), then the
    # timed call on the warm session (see bench_infill)
    warm = _infill_requests(args.c5_requests, args.c5_seq + 256, 7000, n_infill_bars=4)
    torch.cuda.synchronize()
    tw = time.perf_counter()
    _, wst = generation_batch(m, warm, v, all_controls, greedy=True, return_stats=True)
    torch.cuda.synchronize()
    cold = wst["tokens"] / (time.perf_counter() - tw)
    reqs = _infill_requests(args.c5_requests, args.c5_seq, 5000 + 100 * rank, n_infill_bars=4)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, st = generation_batch(m, reqs, v, all_controls, greedy=True, return_stats=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    lat = np.asarray(st["request_latency_s"])
    return {"tokens": st["tokens"], "steps": st["steps"], "seconds": dt, "cold_tokens_per_s": cold,
            "tokens_per_s": st["tokens"] / dt, "requests": len(reqs),
            "mean_src_len": float(np.mean([len(r[0]) for r in reqs])),
            "p50_latency_s": float(np.percentile(lat, 50)),
            "p90_latency_s": float(np.percentile(lat, 90)),
            "ms_per_decode_step": 1000 * st["step_call_s"] / max(1, st["steps"]),
            "roofline": infill_roofline(args, st, 4 if precision == "fp32" else 2),
            "phases_s": dict({k: round(st[k], 4) for k in ("prepare_s", "prefill_s", "decode_s")},
                             **{k: round(v, 4) for k, v in st.get("decode_phases_s", {}).items()})}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args):
    """The oracle (torch-CPU fp32 restatement of the reference path) on the
    GPU box's host, on bounded samples of the same workloads:
      train  — B=2 sequences of the C2 step shape (fwd + bwd);
      infill — the reference's decode algorithm (full recompute of encoder +
               decoder per token, generation.py:209-225,542-545) on one C2
               request with an S>=1024 source, greedy, ~10 s of tokens.
    Threads: torch.set_num_threads(os.cpu_count()) as BASELINE.md asks,
    unless the box pins this job's CPU share in OMP_NUM_THREADS (the GPU box
    does: 16), which is then used and reported."""
    from oracle import ref_cpu
    from smer_music_generation_amd.generation import _prepare
    from smer_music_generation_amd.synth import synth_training_batch
    from smer_music_generation_amd.vocab import WordVocab
    ncpu = os.cpu_count() or 1
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or ncpu
    torch.set_num_threads(threads)
    v = WordVocab(0, CTRL)
    cfg = dict(d_model=args.d_model, nhead=args.nhead, num_encoder_layers=args.layers,
               num_decoder_layers=args.layers)
    sd = ref_cpu.init_params(309, args.d_model, args.ff, args.layers, args.layers, seed=0)
    sd["pos_enc.pe"] = ref_cpu.pe_table(2400, args.d_model)
    B = 2
    b = synth_training_batch(7, v, B, args.seq, args.tgt)
    ref_cpu.train_step(sd, cfg, b, v.control_indices, 0.8, 8)  # warm-up
    t0 = time.perf_counter()
    n = 0
    while True:
        ref_cpu.train_step(sd, cfg, b, v.control_indices, 0.8, 8)
        n += 1
        if time.perf_counter() - t0 > 10.0 or n >= 5:
            break
    dt = time.perf_counter() - t0
    res = {"value": B * (args.seq + args.tgt) * n / dt, "unit": "train tokens/s (B*(S+T))",
           "cores": threads, "os_cpu_count": ncpu, "cpu_model": _cpu_model(), "kind": "port",
           "sample": "%d oracle train steps (fwd+bwd, fp32, torch CPU) at B=%d S=%d T=%d, C2 model"
                     % (n, B, args.seq, args.tgt)}
    # infill: the reference algorithm, full recompute per token
    ev, tracks, bars = _infill_requests(1, args.seq, 4242)[0]
    src, _, _, target, no_whole = _prepare(list(ev), v, tracks, bars)
    fn = ref_cpu.full_recompute_logits_fn(sd, cfg)
    calls = [0]
    t_end = [None]

    class _Budget(Exception):
        pass

    def timed(src_ids, tgt_list):
        if time.perf_counter() > t_end[0]:
            raise _Budget()
        calls[0] += 1
        return fn(src_ids, tgt_list)
    ac = v.density_indices + v.occupation_indices + v.polyphony_indices + v.tensile_indices
    fn(src, [2])  # warm-up
    t0 = time.perf_counter()
    t_end[0] = t0 + 10.0
    try:
        ref_cpu.infill(timed, src, target, v, ac, no_whole, greedy=True)
    except _Budget:
        pass
    dt = time.perf_counter() - t0
    res["infill"] = {"value": calls[0] / dt, "unit": "infill tokens/s (batch 1)", "cores": threads,
                     "kind": "port",
                     "sample": "%d greedy decode tokens of one C2 request (S=%d), full recompute "
                               "per token as generation.py:209-225 (oracle fp32 torch CPU)"
                               % (calls[0], len(src))}
    return res


# every bf16 GEMM tile kernel behind ops.gemm / gemm_wgrad_bias (the calls
# the live HIP-event timer brackets); the split-K reduce is added per call
GEMM_FAMILY = ("gemm_bf16_kernel", "gemm256_bf16_kernel", "gemm256s_bf16_kernel",
               "gemm256_wgrad_kernel", "gemm256s_wgrad_kernel", "gemm64_bf16_kernel",
               "gemm_skinny_bf16_kernel")


def _pmc_traffic():
    """HBM bytes per gemm_bf16_kernel launch (FETCH_SIZE x2 + WRITE_SIZE,
    launch-weighted over the three layout variants) from the newest committed
    rocprofv3 PMC summary (profiles/*_train_pmc_traffic.json, written by
    tools/pmc_traffic.py from tools/profile_round.sh's separate passes)."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                                          "*_train_pmc_traffic.json")))
    if not files:
        return None
    s = json.load(open(files[-1]))
    # the smer_gemm family: 128x128 and 256x256 tile kernels, skinny kernel,
    # split-K slab reduction (one smer_gemm call = tile kernel [+ reduce])
    s = {(k[5:] if k.startswith("void ") else k): v for k, v in s.items()}
    g = [v for k, v in s.items() if k.startswith(GEMM_FAMILY)]
    n = sum(v["launches"] for v in g)
    if not n:
        return None
    red = [v for k, v in s.items() if k.startswith("splitk_reduce_kernel")]
    tot = sum(v["hbm_bytes"] * v["launches"] for v in g + red)
    return {"bytes_per_launch": round(tot / n),
            "source": os.path.basename(files[-1])}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--tgt", type=int, default=256)
    ap.add_argument("--layers", type=int, default=6)
    ap.add_argument("--d-model", dest="d_model", type=int, default=512)
    ap.add_argument("--nhead", type=int, default=8)
    ap.add_argument("--ff", type=int, default=2048)
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--infill-batch", dest="infill_batch", type=int, default=32)
    ap.add_argument("--no-infill", dest="infill", action="store_false")
    ap.add_argument("--no-c5", dest="c5", action="store_false")
    ap.add_argument("--no-c4", dest="c4", action="store_false")
    ap.add_argument("--c4-steps", dest="c4_steps", type=int, default=3)
    ap.add_argument("--c4-warmup", dest="c4_warmup", type=int, default=1)
    ap.add_argument("--c5-requests", dest="c5_requests", type=int, default=64)
    ap.add_argument("--c5-seq", dest="c5_seq", type=int, default=4096)
    ap.add_argument("--no-fp32-infill", dest="fp32_infill", action="store_false",
                    help="skip the fp32 (bit-exact) batched greedy infill lines at C2 and C5")
    ap.add_argument("--no-cpu", dest="cpu", action="store_false")
    ap.add_argument("--no-roofline", dest="roofline", action="store_false")
    ap.add_argument("--grad-wire", dest="grad_wire", choices=("fp32", "bf16"), default="fp32",
                    help="DP gradient all-reduce dtype of the headline step (fp32 = parity)")
    ap.add_argument("--global-batch", dest="global_batch", type=int, default=0,
                    help="strong scaling: fix the GLOBAL batch at this many sequences, split "
                         "evenly over the ranks (default 0: weak scaling, --batch per rank). "
                         "Under DP without it, a 'train_strong' block still reports the step at "
                         "global batch --batch split over the ranks (SURVEY §8e: report both)")
    ap.add_argument("--dry-run", dest="dry_run", action="store_true",
                    help="launcher / DP plumbing check on CPU over gloo (no GPU, no HIP): "
                         "rank-0 broadcast + the bucketed gradient all-reduce, C1 model")
    return ap.parse_args(argv)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """`python bench.py --gpus N` outside torch.distributed.run: start N
    ranks (one per GPU) through torch.distributed.run as a CHILD process and
    exit with its code.  This parent never initialises HIP (no torch.cuda
    call before or after), so the children own the GPUs; rank 0 prints the
    JSON line on the shared stdout."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def per_rank_batch(global_batch, world):
    """Strong scaling: the global batch split evenly over the ranks."""
    if global_batch % world:
        raise SystemExit("--global-batch %d is not divisible by %d ranks" % (global_batch, world))
    return global_batch // world


def scaling_modes(args, world):
    """Both DP scalings of the C2 step: weak = --batch per rank,
    strong = the global batch (--global-batch, else --batch) split over the
    ranks."""
    g = args.global_batch or args.batch
    return {"weak": {"per_rank_batch": args.batch, "global_batch": args.batch * world},
            "strong": {"per_rank_batch": per_rank_batch(g, world), "global_batch": g}}


def dry_run(args, rank, world):
    """Launcher / DP plumbing on CPU (gloo): the C1 model (BASELINE configs[0]
    shapes: 2+2 layers d128) built with a rank-dependent seed, the Trainer's
    rank-0 broadcast, then K timed exchange steps of the real GradBucketer
    (per-layer async SUM all-reduce in backward order) over a rank-dependent
    gradient.  No HIP kernel runs; the line says so (`dry_run`)."""
    from smer_music_generation_amd.model import ScoreTransformer
    from smer_music_generation_amd.train import GradBucketer, Trainer
    from smer_music_generation_amd.vocab import WordVocab
    dev = torch.device("cpu")
    v = WordVocab(0, CTRL)
    torch.manual_seed(100 + rank)  # deliberately different per rank
    m = ScoreTransformer(309, 128, 4, 2, 2, 2048, 2400, 0.0, 0.0)
    tr = Trainer(m, v, grad_wire_dtype=torch.bfloat16 if args.grad_wire == "bf16" else None)
    in_sync = params_in_sync(m, dev, world)
    grad = m.flat_grad()
    bk = GradBucketer(grad, tr._ranges, wire_dtype=tr.grad_wire_dtype)
    order = ["head"] + ["dec%d" % i for i in reversed(range(2))] + \
        ["enc%d" % i for i in reversed(range(2))] + ["embedding"]

    def step():
        grad.fill_(float(rank + 1))
        for name in order:
            bk.reduce(name)
        bk.finish()
        return grad

    dt, g = timed_steps(step, args.steps, args.warmup, dev, world)
    dt = max_over_ranks(dt, dev, world)
    want = world * (world + 1) / 2
    return {"seconds": dt, "params_in_sync_at_init": in_sync,
            "allreduce_ok": bool(torch.all(g == want).item()),
            "bytes_per_step": grad.numel() * (2 if args.grad_wire == "bf16" else 4),
            # the gradient exchange is the same in both modes (one flat buffer
            # of parameters); what changes is the per-rank batch
            "scaling_modes": scaling_modes(args, world)}


def data_feed(per_gpu_tokens_per_s, seconds=3.0):
    """Host side of the training input: one process's rate of
    the pretraining pipeline (stack_batches groups -> span masking -> collate,
    control mode 2) in the trainer's unit, and the worker processes one GPU
    needs at the measured train rate."""
    import math as _m
    from smer_music_generation_amd.data import measure_rate
    r = measure_rate(seconds, 2, True)
    f = measure_rate(seconds / 2, 2, False)
    need = per_gpu_tokens_per_s / r["tokens_per_s"]
    return {"metric": "pretraining items + collate, collated B*(S+T) tokens/s per host process",
            "value": round(r["tokens_per_s"], 1), "finetune_value": round(f["tokens_per_s"], 1),
            "ids_per_s": round(r["ids_per_s"], 1), "processes_per_gpu": _m.ceil(need),
            "train_tokens_per_s_per_gpu": round(per_gpu_tokens_per_s, 1),
            "source": "synthetic corpus (240 songs, 8-24 bars), max_token_length 2200"}


def main():
    args = parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print("bench: --gpus %d but WORLD_SIZE=%d; reporting the real world size"
              % (args.gpus, world), file=sys.stderr)
    if args.dry_run:
        if world > 1:
            dist.init_process_group("gloo")
        r = dry_run(args, rank, world)
        if rank == 0:
            print(json.dumps({
                "metric": "launcher dry run (DP plumbing on CPU, no GPU work; not a measurement)",
                "value": None, "unit": "s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(1000 * r["seconds"] / args.steps, 3),
                "higher_is_better": False, "scaling": "weak", "vs_baseline": None,
                "dtype": args.grad_wire, "data": "synthetic", "dry_run": True,
                "config": {"workload": "C1 model, rank-0 broadcast + bucketed gradient "
                                       "all-reduce (gloo)", "parallelism": "dp%d" % world},
                "params_in_sync_at_init": r["params_in_sync_at_init"],
                "allreduce_ok": r["allreduce_ok"], "bytes_per_step": r["bytes_per_step"],
                "scaling_modes": r["scaling_modes"]}))
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    from smer_music_generation_amd import _lib
    _lib.load()

    wire = torch.bfloat16 if args.grad_wire == "bf16" else None
    strong = args.global_batch > 0
    if strong:  # the headline itself at a fixed global batch
        import copy
        head = copy.copy(args)
        head.batch = per_rank_batch(args.global_batch, world)
    else:
        head = args
    tr = bench_train(head, dev, rank, world, grad_wire=wire)
    # DP, weak headline: the strong-scaling step beside it (global batch
    # --batch split over the ranks), SURVEY §8e "report both"
    tr_strong = None
    if world > 1 and not strong:
        import copy
        a = copy.copy(args)
        a.roofline = False
        a.batch = per_rank_batch(args.batch, world)
        tr_strong = bench_train(a, dev, rank, world, grad_wire=wire)
    # DP only: the same step with the opt-in bf16 gradient all-reduce
    # (half the xGMI bytes), reported beside the fp32 (parity) headline
    tr_alt = None
    if world > 1 and wire is None:
        import copy
        a = copy.copy(head)
        a.roofline = False
        tr_alt = bench_train(a, dev, rank, world, grad_wire=torch.bfloat16)
    c4 = bench_train_c4(args, dev, rank, world, "fp8") if args.c4 else None
    c4b = bench_train_c4(args, dev, rank, world, "bf16") if args.c4 else None
    inf = None
    if args.infill:
        inf = bench_infill(args, dev, rank)
        if world > 1:
            t = torch.tensor([inf["tokens"], inf["seconds"]], device=dev, dtype=torch.float64)
            tok = t[0:1].clone()
            dist.all_reduce(tok)
            sec = t[1:2].clone()
            dist.all_reduce(sec, op=dist.ReduceOp.MAX)
            inf["tokens_per_s"] = tok.item() / sec.item()
    b1 = bench_infill_batch1(args, dev, rank) if args.infill else None
    c5 = None
    if args.infill and args.c5:
        c5 = bench_infill_c5(args, dev, rank)
        if world > 1:
            t = torch.tensor([c5["tokens"]], device=dev, dtype=torch.float64)
            dist.all_reduce(t)
            sec = torch.tensor([c5["seconds"]], device=dev, dtype=torch.float64)
            dist.all_reduce(sec, op=dist.ReduceOp.MAX)
            c5["tokens_per_s"] = t.item() / sec.item()
    # the bit-exact decode path (fp32; greedy ids equal the reference's),
    # same requests and method as the bf16 lines above
    inf32 = c5_32 = None
    if args.infill and args.fp32_infill:
        torch.cuda.empty_cache()
        inf32 = bench_infill(args, dev, rank, "fp32")
        if args.c5:
            torch.cuda.empty_cache()
            c5_32 = bench_infill_c5(args, dev, rank, "fp32")
        torch.cuda.empty_cache()
    cpu = cpu_baseline(args) if (args.cpu and rank == 0 and world == 1) else None
    feed = data_feed(tr["tokens_per_s"] / world) if (args.cpu and rank == 0) else None

    if rank == 0:
        roof = None
        if "gemm" in tr:
            g = tr["gemm"]
            roof = {"bound": "mfma",
                    "kernel": "smer_gemm family (%s + splitk_reduce_kernel): achieved, frac "
                              "and traffic all over this set" % ", ".join(GEMM_FAMILY),
                    "achieved": round(g["tflops"], 2), "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(g["tflops"] / BF16_PEAK_TFLOPS, 4), "traffic": (_pmc_traffic() or {}).get("bytes_per_launch"),
                    "traffic_unit": "HBM bytes per launch (rocprofv3 PMC)",
                    "traffic_source": (_pmc_traffic() or {}).get("source"),
                    "avg_launch_us": round(g["avg_us"], 2),
                    "flops_per_launch": g["flops_per_launch"],
                    "share_of_step_time": round(g["share_of_step"], 3)}
        line = {
            "metric": "infill tokens/sec + train tokens/sec, SMER seq_len=1024, 1/2/4/8 MI355X",
            "value": round(tr["tokens_per_s"], 1), "unit": "train tokens/s (B*(S+T))",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(tr["ms_per_step"], 3), "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic SMER-grammar token batches (seeded), random xavier_normal weights",
            "config": {"workload": "C2 train step: 6+6 layers d512 h8 ff2048 V309, per-GPU "
                                   "B=%d S=%d T=%d, dropout %.1f, fused WCE + Adam%s"
                                   % (head.batch, args.seq, args.tgt, args.dropout,
                                      " + RCCL grad all-reduce" if world > 1 else ""),
                       "global_batch": head.batch * world, "seq_len": args.seq,
                       "tgt_len": args.tgt, "parallelism": "dp%d" % world},
            "train": {k: (round(val, 4) if isinstance(val, float) else val)
                      for k, val in tr.items() if k != "gemm"},
            "train_strong": tr_strong and {
                "scaling": "strong", "global_batch": args.batch,
                "per_rank_batch": args.batch // world,
                "tokens_per_s": round(tr_strong["tokens_per_s"], 1),
                "ms_per_step": round(tr_strong["ms_per_step"], 3),
                "note": "same step at a fixed global batch split over the ranks (the headline "
                        "is weak scaling: B per rank)"},
            "train_bf16_allreduce": tr_alt and {
                "tokens_per_s": round(tr_alt["tokens_per_s"], 1),
                "ms_per_step": round(tr_alt["ms_per_step"], 3),
                "note": "same step, DP gradient all-reduce in bf16 (opt-in; fp32 is the parity "
                        "default)"},
            "roofline": roof,
            "infill": inf and {"metric": "infill tokens/s (greedy, KV-cached, batched; warm "
                                         "decode session)",
                               "value": round(inf["tokens_per_s"], 1),
                               "cold_value": round(inf["cold_tokens_per_s"], 1),
                               "requests_per_gpu": inf["requests"],
                               "mean_src_len": round(inf["mean_src_len"], 1),
                               "decode_steps": inf["steps"], "tokens": inf["tokens"],
                               "ms_per_decode_step": round(inf["ms_per_decode_step"], 3),
                               "roofline": inf["roofline"],
                               "phases_s": inf["phases_s"], "cold_phases_s": inf["cold_phases_s"],
                               "parallelism": "replicas",
                               "batch1": b1 and dict(b1, metric="plugin call generation_all "
                                                     "(batch 1, default weighted sampling, "
                                                     "KV-cached), tokens/s")},
            "train_c4": c4 and {"metric": "C4 train tokens/s (B*(S+T)), 12+12 layers d768 h12, "
                                          "S=2048 T=512",
                                "dtype": "fp8 (e4m3 forward GEMMs: QKV (layers >= 1), "
                                         "attention out-projections, FFN1, FFN2, cross-attention "
                                         "Q and K/V; e4m3 dgrads: FFN2, FFN1, out-projections, "
                                         "QKV, cross Q, memory; e4m3 weight + bias gradients: "
                                         "the same Linears; delayed per-tensor scaling; "
                                         "FFN1's output, dh and the dropped LayerNorm "
                                         "gradients stored in e4m3 only; attention, the first "
                                         "layers' QKV and the vocab head bf16)",
                                "value": round(c4["tokens_per_s"], 1),
                                "ms_per_step": round(c4["ms_per_step"], 2),
                                "step_tflops_per_gpu": round(c4["step_tflops_per_gpu"], 1),
                                "frac_of_fp8_peak": round(c4["step_tflops_per_gpu"] / FP8_PEAK_TFLOPS, 4),
                                "frac_of_bf16_peak": round(c4["mfma_frac_whole_step"], 4),
                                "bf16_value": c4b and round(c4b["tokens_per_s"], 1),
                                "bf16_ms_per_step": c4b and round(c4b["ms_per_step"], 2),
                                "global_batch": args.batch * world, "steps": args.c4_steps,
                                "parallelism": "dp%d" % world},
            "infill_c5": c5 and {"metric": "C5 batched infill tokens/s (64 requests x ~4096-token "
                                           "sources, 4 bars of one track each, greedy; warm "
                                           "decode session)",
                                 "value": round(c5["tokens_per_s"], 1),
                                 "cold_value": round(c5["cold_tokens_per_s"], 1),
                                 "p50_latency_s": round(c5["p50_latency_s"], 4),
                                 "p90_latency_s": round(c5["p90_latency_s"], 4),
                                 "ms_per_decode_step": round(c5["ms_per_decode_step"], 3),
                                 "requests_per_gpu": c5["requests"],
                                 "mean_src_len": round(c5["mean_src_len"], 1),
                                 "decode_steps": c5["steps"], "tokens": c5["tokens"],
                                 "roofline": c5["roofline"],
                                 "phases_s": c5["phases_s"], "parallelism": "replicas"},
            "infill_fp32": inf32 and {
                "metric": "infill tokens/s on the bit-exact fp32 decode path (greedy ids equal "
                          "the reference's), C2 requests as `infill`, warm session",
                "value": round(inf32["tokens_per_s"], 1),
                "cold_value": round(inf32["cold_tokens_per_s"], 1),
                "ms_per_decode_step": round(inf32["ms_per_decode_step"], 3),
                "decode_steps": inf32["steps"], "tokens": inf32["tokens"],
                "roofline": inf32["roofline"], "phases_s": inf32["phases_s"],
                "per_rank": True},
            "infill_c5_fp32": c5_32 and {
                "metric": "C5 batched infill tokens/s on the bit-exact fp32 decode path, "
                          "requests as `infill_c5`, warm session",
                "value": round(c5_32["tokens_per_s"], 1),
                "cold_value": round(c5_32["cold_tokens_per_s"], 1),
                "p50_latency_s": round(c5_32["p50_latency_s"], 4),
                "ms_per_decode_step": round(c5_32["ms_per_decode_step"], 3),
                "decode_steps": c5_32["steps"], "tokens": c5_32["tokens"],
                "roofline": c5_32["roofline"], "phases_s": c5_32["phases_s"],
                "per_rank": True},
            "cpu_baseline": cpu,
            "data_pipeline": feed,
        }
        print(json.dumps(line))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
