#!/usr/bin/env python3
"""Benchmark: 1024x1024 images/sec through the W4A16 (GPTQ int4) ViT-H SAM image encoder.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--model vit_h]

One process per GPU (for N > 1 launched by ``torch.distributed.run``; RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_* from the env).  A "step" = one encoder forward over the per-GPU batch of
synthetic images already resident in HBM (a HIP-graph replay of the fused engine).  Weights are
random-init ViT-H, RTN-quantised into the reference's packed int4 format on rank 0 and RCCL-
broadcast to the other ranks (the only collective on the data path).  Per-GPU work is fixed
("weak" scaling): batch 4 per GPU at N=1 (BASELINE config 3), 8 per GPU at N>1 (config 4 at
N=8 = global batch 64).

Besides the throughput line, it reports for the dominant kernel (all W4A16 GEMM launches of one
forward) its live roofline fraction from HIP events on the launch stream, and the CPU baseline:
the oracle restatement of the reference's fp32 CPU fake-quant path on one image (rank 0, N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "sam-quantization_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "1024×1024 images/sec through quantized ViT-H encoder; % of MFMA/HBM roofline"
PEAK_FP16_TFLOPS = 2500.0   # MI355X dense fp16/bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def gemm_roofline(eng, bufs_batch: int, reps: int = 3):
    """Average duration of every W4A16 GEMM launch of one forward, measured with HIP events on
    the launch stream; achieved = algorithmic FLOPs (2*M*N*K per launch) / duration."""
    from samq import ops
    bufs = eng.buffers(bufs_batch)
    stream = torch.cuda.current_stream()
    rows = bufs["x"].numel() // bufs["x"].shape[-1]
    records = []
    for _ in range(reps):
        for p in eng.plans:
            for lin, a, out, epi in ((p.qkv, bufs["xn"], bufs["qkv"], ops.EPI_BIAS),
                                     (p.proj, bufs["att"], bufs["x"], ops.EPI_RESADD_F32),
                                     (p.lin1, bufs["xn"], bufs["hid"], ops.EPI_BIAS_GELU),
                                     (p.lin2, bufs["hid"], bufs["x"], ops.EPI_RESADD_F32)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                lin.forward_epilogue(a, epi, out=out)
                e1.record(stream)
                records.append((e0, e1, 2.0 * rows * lin.infeatures * lin.outfeatures))
    torch.cuda.synchronize()
    t = sum(e0.elapsed_time(e1) for e0, e1, _ in records) / 1e3
    flops = sum(f for *_, f in records)
    n = len(records)
    achieved = flops / t / 1e12
    return dict(bound="mfma", achieved=round(achieved, 1), peak=PEAK_FP16_TFLOPS, unit="TFLOP/s",
                frac=round(achieved / PEAK_FP16_TFLOPS, 4), traffic=None,
                kernel="w4a16_gemm_kernel (all 4 ViT-H projection shapes)", launches_timed=n,
                avg_launch_us=round(t / n * 1e6, 2))


def cpu_baseline(model_name: str):
    """Oracle restatement of the reference CPU fake-quant path (fp32 encoder with dequantised
    int4 weights), one 1024x1024 image, rank 0 only."""
    sys.path.insert(0, str(REPO))
    from oracle import sam_ref, synth
    threads = len(os.sched_getaffinity(0))
    threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))
    torch.set_num_threads(threads)
    cfg = synth.encoder_config(model_name)
    g = torch.Generator().manual_seed(0)
    st = {}
    for k, shape in _state_shapes(cfg).items():
        st[k] = torch.randn(shape, generator=g) * 0.02
    o = sam_ref.EncoderOracle(cfg, st)
    img = torch.randn(1, 3, 1024, 1024, generator=g)
    t0 = time.perf_counter()
    o(img)
    dt = time.perf_counter() - t0
    return dict(value=round(1.0 / dt, 4), unit="img/s", cores=threads, kind="port",
                sample=f"1 image, {model_name} fp32 CPU fake-quant op graph (oracle/sam_ref.py), "
                       f"{dt:.1f} s wall, torch {threads} threads, CPU: {_cpu_model()}")


def _state_shapes(cfg):
    shapes = {}
    c, heads = cfg["embed_dim"], cfg["num_heads"]
    hd = c // heads
    grid = cfg["img_size"] // 16
    shapes["patch_embed.proj.weight"] = (c, 3, 16, 16)
    shapes["patch_embed.proj.bias"] = (c,)
    shapes["pos_embed"] = (1, grid, grid, c)
    for i in range(cfg["depth"]):
        pre = f"blocks.{i}."
        side = grid if i in cfg["global_attn_indexes"] else 14
        for n, s in (("norm1.weight", (c,)), ("norm1.bias", (c,)), ("attn.qkv.weight", (3 * c, c)),
                     ("attn.qkv.bias", (3 * c,)), ("attn.proj.weight", (c, c)), ("attn.proj.bias", (c,)),
                     ("attn.rel_pos_h", (2 * side - 1, hd)), ("attn.rel_pos_w", (2 * side - 1, hd)),
                     ("norm2.weight", (c,)), ("norm2.bias", (c,)), ("mlp.lin1.weight", (4 * c, c)),
                     ("mlp.lin1.bias", (4 * c,)), ("mlp.lin2.weight", (c, 4 * c)), ("mlp.lin2.bias", (c,))):
            shapes[pre + n] = s
    shapes.update({"neck.0.weight": (256, c, 1, 1), "neck.1.weight": (256,), "neck.1.bias": (256,),
                   "neck.2.weight": (256, 256, 3, 3), "neck.3.weight": (256,), "neck.3.bias": (256,)})
    return shapes


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=0, help="images per GPU (default 4 at N=1, 8 at N>1)")
    ap.add_argument("--model", default="vit_h")
    ap.add_argument("--groupsize", type=int, default=-1)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    from samq import dist as sdist
    from samq.synthetic import flops_per_image, random_quant_encoder

    rank, world = sdist.init_from_env()
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using {world}")
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    batch = args.batch or (4 if world == 1 else 8)

    t0 = time.time()
    enc = random_quant_encoder(args.model, args.groupsize, device=dev, init=(rank == 0))
    nbytes = sdist.broadcast_state(enc, src=0)
    eng = enc.engine()
    log(f"[rank {rank}] model ready in {time.time() - t0:.1f}s (broadcast {nbytes / 1e6:.1f} MB)")

    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    img = torch.randn((batch, 3, 1024, 1024), generator=g, device=dev, dtype=torch.float16)
    if args.no_graph:
        run = lambda: eng(img)  # noqa: E731
    else:
        graph, _ = eng.capture(img)
        run = graph.replay
    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()

    roof = gemm_roofline(eng, batch)
    fl = flops_per_image(enc)
    total_imgs = world * batch * args.steps
    value = total_imgs / elapsed
    if rank == 0:
        e2e_tflops = value / world * fl["total"] / 1e12
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "img/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp16", "data": "synthetic",
            "config": {"workload": f"SAM {args.model} image encoder W4A16 GPTQ (int4 RTN-packed, "
                                   f"groupsize {args.groupsize}), {batch} x 1024x1024 images per GPU",
                       "model": args.model, "global_batch": world * batch, "per_gpu_batch": batch,
                       "seq_len": 4096, "parallelism": f"image-parallel x{world} (weights RCCL-broadcast once)",
                       "graph": not args.no_graph},
            "roofline": roof,
            "e2e": {"tflop_per_image": round(fl["total"] / 1e12, 4), "achieved_tflops_per_gpu": round(e2e_tflops, 1),
                    "frac_of_fp16_peak": round(e2e_tflops / PEAK_FP16_TFLOPS, 4),
                    "frac_of_int8_peak": round(e2e_tflops / (2 * PEAK_FP16_TFLOPS), 4)},
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.model)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
