#!/usr/bin/env python3
"""Benchmark of the two hot paths (BASELINE.json metric:
"RQ-VAE items encoded/s + SASRec seqs scored/s @1/8 GPU").

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Primary line (``value``): RQ-VAE encode, config C2 = 3x256 codebooks, in 768 -> [256,128] -> e 32,
100k synthetic items per rank per step (``RQVAE.get_indices`` on device-resident inputs).  Items
shard across ranks with no collective ("scaling": "weak").  The SASRec scoring config C3 (2 blocks,
d 64, n 50, 100k-item catalog, B users per rank per step, ``SASRec.predict``) is reported in the
same JSON line under "sasrec".  Rank 0 also times the CPU oracle (oracle/) on a bounded sample of
the same workload ("cpu_baseline").
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import gr_amd  # noqa: E402
from gr_amd import synth  # noqa: E402

METRIC = "RQ-VAE items encoded/s + SASRec seqs scored/s @1/8 GPU; HR@10/NDCG@10 parity"
FP32_PEAK_TFLOPS = 157.3      # MI355X fp32 matrix (= vector) peak, MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0

# Algorithmic work per unit (SURVEY §8d / DESIGN.md)
RQ_IN, RQ_LAYERS, RQ_E, RQ_L, RQ_K = 768, (256, 128), 32, 3, 256
RQ_FLOP_PER_ITEM = 2 * (768 * 256 + 256 * 128 + 128 * 32) + 2 * RQ_L * RQ_K * RQ_E   # 516,096
RQ_BYTES_PER_ITEM = 768 * 4 + RQ_L * 8                                                # 3,096
SAS_D, SAS_N, SAS_ITEMS, SAS_MLP, SAS_BLOCKS = 64, 50, 100_000, 64, 2


def sas_flop_per_user(d=SAS_D, n=SAS_N, items=SAS_ITEMS, mlp=SAS_MLP, blocks=SAS_BLOCKS):
    """Reference formulation (dead W_Q/K/V excluded): per block in-proj 2*n*d*3d, scores and P.V
    2*2*n*n*d, out-proj 2*n*d*d, FFN 2*2*n*d*mlp; scoring 2*d*(items+1)."""
    per_block = 2 * n * d * 3 * d + 4 * n * n * d + 2 * n * d * d + 4 * n * d * mlp
    return blocks * per_block + 2 * d * (items + 1)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rq-items", type=int, default=100_000)
    ap.add_argument("--sas-batch", type=int, default=2048)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="budget per CPU baseline leg")
    ap.add_argument("--skip-sasrec", action="store_true")
    return ap.parse_args()


def timed(fn, steps, warmup, world):
    """W untimed steps, then exactly K steps between barrier+synchronize; returns (max-over-ranks
    wall seconds, mean device ms per step from HIP events on the launch stream)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    dev_ms = sum(s.elapsed_time(e) for s, e in ev) / steps
    if world > 1:
        t = torch.tensor([wall], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    return wall, dev_ms


def cpu_threads():
    n = len(os.sched_getaffinity(0))
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", n))))


def cpu_rq_baseline(model, budget_s):
    """Oracle restatement of get_indices (oracle/rq_oracle.py) on host cores: 100k-item batches of
    the same synthetic workload, repeated until ~budget_s."""
    from oracle import rq_oracle
    torch.set_num_threads(cpu_threads())
    lin = model.encoder.linears()
    ws = [l.weight.detach().cpu() for l in lin]
    bs = [l.bias.detach().cpu() for l in lin]
    cbs = [c.cpu() for c in model.rq.codebooks()]
    x = synth.items(100_000, 12345, "cuda").cpu()
    rq_oracle.get_indices(x[:4096], ws, bs, cbs)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s or n == 0:
        rq_oracle.get_indices(x, ws, bs, cbs)
        n += x.shape[0]
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "items/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"oracle/rq_oracle.get_indices on {n} synthetic C2 items (100k per call, "
                      f"{dt:.1f} s, fp32 torch CPU)"}


def cpu_sas_baseline(model, budget_s):
    from oracle import sasrec_oracle
    torch.set_num_threads(cpu_threads())
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    seqs = synth.sequences(128, SAS_N, SAS_ITEMS, 777, "cuda").cpu()
    sasrec_oracle.predict(seqs[:8], sd, SAS_BLOCKS, 1, 1e-8)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s or n == 0:
        sasrec_oracle.predict(seqs, sd, SAS_BLOCKS, 1, 1e-8)
        n += seqs.shape[0]
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "seqs/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"oracle/sasrec_oracle.predict, {n} users in batches of 128 (C3 shapes, "
                      f"{dt:.1f} s)"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world:
        if world == 1 and a.gpus > 1:
            sys.exit("bench.py: --gpus N>1 must be launched with torch.distributed.run (one rank per GPU)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    # ---------------- RQ-VAE encode, config C2 (items shard over ranks: per-rank batch fixed)
    rq_model = synth.rqvae_model(RQ_L, RQ_K, dev)
    x = synth.items(a.rq_items, 1000 + rank, dev)
    rq_wall, rq_dev_ms = timed(lambda: rq_model.get_indices(x), a.steps, a.warmup, world)
    items_total = a.rq_items * world * a.steps
    rq_value = items_total / rq_wall
    achieved_tf = RQ_FLOP_PER_ITEM * a.rq_items / (rq_dev_ms * 1e-3) / 1e12
    line = {
        "metric": METRIC, "value": rq_value, "unit": "items/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": rq_wall / a.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": "rq_c2: RQ-VAE get_indices, 3x256 codebooks, in 768 -> [256,128] -> "
                               "e 32, data-derived codebooks",
                   "items_per_rank_per_step": a.rq_items, "global_batch": a.rq_items * world,
                   "parallelism": f"item-sharded x{world}, no collective"},
        "roofline": {"bound": "mfma", "achieved": achieved_tf, "peak": FP32_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved_tf / FP32_PEAK_TFLOPS, "traffic": None,
                     "kernel": "gr_rq_encode_f32 (encoder linears + quantize, per call)",
                     "flop_per_unit": RQ_FLOP_PER_ITEM, "units_per_launch": a.rq_items,
                     "device_ms_per_launch": rq_dev_ms,
                     "hbm_algorithmic_GBs": RQ_BYTES_PER_ITEM * a.rq_items / (rq_dev_ms * 1e-3) / 1e9},
    }
    # ---------------- SASRec predict, config C3 (users shard over ranks)
    if not a.skip_sasrec:
        p = synth.sasrec_params(SAS_D, SAS_N, SAS_BLOCKS, 1, SAS_MLP, dev)
        sas_model = synth.sasrec_model(SAS_ITEMS, p, dev)
        seqs = synth.sequences(a.sas_batch, SAS_N, SAS_ITEMS, 2000 + rank, dev)
        out = torch.empty((a.sas_batch, SAS_ITEMS + 1), dtype=torch.float32, device=dev)
        binding = gr_amd.ops.SasrecBinding(sas_model)
        sas_wall, sas_dev_ms = timed(lambda: gr_amd.ops.sasrec_predict(binding, seqs, out=out),
                                     a.steps, a.warmup, world)
        users = a.sas_batch * world * a.steps
        fl = sas_flop_per_user()
        tf = fl * a.sas_batch / (sas_dev_ms * 1e-3) / 1e12
        line["sasrec"] = {
            "metric": "seqs_scored/s", "value": users / sas_wall, "unit": "seqs/s",
            "ms_per_step": sas_wall / a.steps * 1e3,
            "config": {"workload": "sas_c3: SASRec predict, 2 blocks, d 64, n 50, H 1, mlp 64, "
                                   "100k-item full-catalog logits", "users_per_rank_per_step": a.sas_batch},
            "roofline": {"bound": "mfma", "achieved": tf, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": tf / FP32_PEAK_TFLOPS, "flop_per_unit": fl,
                         "kernel": "gr_sasrec_predict_f32 (per call)", "device_ms_per_launch": sas_dev_ms,
                         "logits_write_GBs": a.sas_batch * (SAS_ITEMS + 1) * 4 / (sas_dev_ms * 1e-3) / 1e9},
        }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        line["cpu_baseline"] = cpu_rq_baseline(rq_model, a.cpu_seconds)
        if not a.skip_sasrec:
            line["sasrec"]["cpu_baseline"] = cpu_sas_baseline(sas_model, a.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
