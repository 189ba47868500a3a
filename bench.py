#!/usr/bin/env python3
"""Benchmark of the two hot paths (BASELINE.json metric:
"RQ-VAE items encoded/s + SASRec seqs scored/s @1/8 GPU; HR@10/NDCG@10 parity").

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

``python bench.py --gpus N`` (N > 1) outside torch.distributed.run launches its N ranks itself: the
parent imports neither torch nor gr_amd, runs ``torch.distributed.run`` as a child process (one rank
per GPU, rendezvous on 127.0.0.1), relays rank 0's JSON line and exits with the children's status.

Primary line (``value``): RQ-VAE encode at config C2 = 3x256 codebooks, in 768 -> [256,128] -> e 32,
100k synthetic items per rank per step (``RQVAE.get_indices`` on device-resident inputs).  Items
shard across ranks with no collective ("scaling": "weak").  The same JSON line carries:
  * "sasrec"    — C3: SASRec.predict, 2 blocks, d 64, n 50, 100k-item catalog, logits written
                  (users shard across ranks, no collective), plus the fused rank path (no logits);
  * "rq_c4"     — C4: 4x1024 codebooks, a fixed 10M-item catalog split over the ranks (strong);
  * "sasrec_c5" — C5: d 128, n 200, 1M-item catalog sharded over the ranks: users' hidden states
                  all-gathered, every rank scores its catalog shard, strict-'>' counts all-reduced
                  and per-shard top-10 all-gathered over RCCL; 512 users per rank (B = 512 N, weak
                  scaling: each rank forwards 512 sequences and scores B users x 1/N of the catalog);
  * "ref_eval"  — SASRec/evaluate.py at the reference's own configuration (d 16, n 20, 706 items,
                  95,423 users in batches of 128);
  * "c5_rank"   — one rank's step of the N = 8 C5 point on one GPU (forward of its 512 users,
                  target logits + fused rank/top-10 of all 4096 users on a 125k-row shard, merge of
                  the 8 x 10 candidates), with the per-kernel split.
Each "roofline" is for the DOMINANT kernel of its path, timed alone with HIP events on the launch
stream; "traffic" (HBM bytes per launch) comes from the committed rocprofv3 PMC summary
(profiles/traffic.json, FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM).  Rank 0 at N=1 also
times the CPU oracle (oracle/) on a bounded sample of the same workloads ("cpu_baseline").
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time


def _self_launch():
    """``--gpus N`` (N > 1) outside torch.distributed.run: start the N ranks as a child
    ``python -m torch.distributed.run`` and return its exit status (None: run in this process).
    Nothing here touches the GPU (no torch import), so the parent never holds a device context."""
    if "WORLD_SIZE" in os.environ or "LOCAL_RANK" in os.environ:
        return None
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    known, _ = ap.parse_known_args()
    if known.gpus <= 1:
        return None
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:   # a free rendezvous port
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC: RCCL across processes
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={known.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=env).returncode


if __name__ == "__main__":
    _rc = _self_launch()
    if _rc is not None:
        sys.exit(_rc)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import gr_amd  # noqa: E402
from gr_amd import ops, synth  # noqa: E402

METRIC = "RQ-VAE items encoded/s + SASRec seqs scored/s @1/8 GPU; HR@10/NDCG@10 parity"
FP32_PEAK_TFLOPS = 157.3      # MI355X fp32 matrix (= vector) peak, MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0

# Algorithmic work per unit (SURVEY §8d / DESIGN.md §4)
ENC_FLOP_PER_ITEM = 2 * (768 * 256 + 256 * 128 + 128 * 32)          # 466,944: encoder MLP


def rq_flop_per_item(L, K, e=32):
    return ENC_FLOP_PER_ITEM + 2 * L * K * e                          # C2: 516,096


def rq_bytes_per_item(L):
    return 768 * 4 + L * 8                                            # C2: 3,096


def sas_flop_per_user(d, n, items, mlp=64, blocks=2):
    """Reference formulation (dead W_Q/K/V excluded): per block in-proj 2*n*d*3d, scores and P.V
    2*2*n*n*d, out-proj 2*n*d*d, FFN 2*2*n*d*mlp; scoring 2*d*(items+1)."""
    per_block = 2 * n * d * 3 * d + 4 * n * n * d + 2 * n * d * d + 4 * n * d * mlp
    return blocks * per_block + 2 * d * (items + 1)


def sas_exec_flop_per_user(d, n, items, mlp=64, blocks=2, causal=True, tail_h=False, heads=1):
    """Flops the kernels execute per user: every block but the last in full,
    attention over the causal n(n+1)/2 query-key pairs (``causal``; the one-wave C3 kernel computes
    the whole n x n tile, ``causal=False``); the last block at position n-1 only (q, one query's
    attention, out-proj, FFN) plus, in the K|V form, the K|V projection of all n tokens -- the
    H-form tail (``tail_h``, sas_tail_h2_kernel) instead computes W_k^T q and W_v u (2 d^2 each)
    and dots every head's d-vector with the n LayerNorm rows (4 n d per head); scoring
    2*d*(items+1) (``items`` = -1: forward only)."""
    pairs = n * (n + 1) // 2 if causal else n * n
    full = 2 * n * d * 3 * d + 4 * pairs * d + 2 * n * d * d + 4 * n * d * mlp
    if tail_h:
        last = 2 * d * d + 2 * d * d + 4 * n * d * heads + 2 * d * d + 2 * d * d + 4 * d * mlp
    else:
        last = 2 * n * d * 2 * d + 2 * d * d + 4 * n * d + 2 * d * d + 4 * d * mlp
    return (blocks - 1) * full + last + 2 * d * (items + 1)


# device of the bench's own small collectives: "cuda" (RCCL, or gloo on device tensors in the
# rehearsal mode); "cpu" for the launcher self-test (GR_BENCH_DEVICE=cpu, no GPU needed)
COLL_DEV = "cuda"

# C5 at N > 1: the split exchange's user sub-batches per step (dist.sharded_rank_topk_batches),
# from the c5_rank leg's overlapped_ms_p2 / _p4 figures (P = 4 scores in launches too small)
C5_PIPELINE_DEFAULT = 2
# the exchange forms bench_sas_c5's auto mode times at N > 1 (make_step)
C5_EXCHANGES = ("serial", "split", "xstep")


def per_rank(x, world):
    """``x`` (this rank's float) from every rank, in rank order (a collective at world > 1)."""
    if world <= 1 or not dist.is_initialized():
        return [x]
    t = torch.zeros(world, dtype=torch.float64, device=COLL_DEV)
    t[dist.get_rank()] = x
    dist.all_reduce(t)
    return t.tolist()


def result_checksum(res, world):
    """a digest of the merged C5 result (1-based ranks, top-k values and ids, all
    [B]-sized and identical on every rank after the exchange), gathered from every rank so the line
    shows the ranks agreed.  For the same users it is independent of the world size: B = c5_batch x N,
    so N = 1 with --c5-batch 4096 reproduces the N = 8 digest (profiles/r06/c5_digest_world_independence.txt)."""
    import hashlib
    rk, v, i = res
    hsh = hashlib.sha256()
    for t in (rk.to(torch.int64), v.to(torch.float32), i.to(torch.int64)):
        hsh.update(t.contiguous().cpu().numpy().tobytes())
    dg = hsh.hexdigest()[:16]
    mine = int(dg, 16) & ((1 << 62) - 1)
    allr = [mine]
    if world > 1 and dist.is_initialized():
        t = torch.zeros(world, dtype=torch.int64, device=COLL_DEV)
        t[dist.get_rank()] = mine
        dist.all_reduce(t)
        allr = t.tolist()
    return {"sha256_16": dg, "ranks_agree": all(c == mine for c in allr), "n_ranks_reporting": len(allr),
            "sum_rank": int(rk.to(torch.int64).sum()), "hr10": float((rk <= 10).double().mean()),
            "topk_id_sum": int(i.to(torch.int64).sum())}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rq-items", type=int, default=100_000)
    ap.add_argument("--sas-batch", type=int, default=2048)
    ap.add_argument("--c4-items", type=int, default=10_000_000)
    ap.add_argument("--c5-batch", type=int, default=512,
                    help="C5 users PER RANK per step: B = c5_batch x N users, so every rank forwards "
                         "c5_batch sequences and scores B users against its 1/N of the catalog")
    ap.add_argument("--c5-rank-world", type=int, default=8,
                    help="c5_rank leg: the world size whose per-rank step it times on one GPU")
    ap.add_argument("--c5-items", type=int, default=1_000_000)
    ap.add_argument("--c5-exchange", default="auto", choices=("auto",) + C5_EXCHANGES,
                    help="C5 exchange form at N > 1: serial; split (--c5-pipeline user sub-batches, each "
                         "one's exchange under the next one's scoring); xstep (the exchange under the next "
                         "step's forward); auto: the fastest, timed on a few steps (serial at N = 1)")
    ap.add_argument("--c5-pipeline", type=int, default=C5_PIPELINE_DEFAULT,
                    help="user sub-batches per step of the split exchange")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--train-batch", type=int, default=128, help="sas_train leg: users per rank per step")
    ap.add_argument("--legs", default="", help="comma list of legs to run (default: " + ",".join(LEGS) + "; also " + ",".join(OPT_LEGS) + ")")
    ap.add_argument("--skip", default="", help="comma list of legs to skip")
    ap.add_argument("--spinup-s", type=float, default=1.0,
                    help="untimed seconds of each leg's workload before its warmup (clock ramp)")
    return ap.parse_args()


def sync_all(world):
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


SPINUP_S = 1.0   # seconds of untimed work before each leg's warmup (set by --spinup-s)


def spinup(fn, seconds=None, world=1):
    """Run ``fn`` untimed for about ``seconds``: MI355X ramps its clocks over the first ~0.1-0.3 s of
    sustained load (measured: the C3 scoring kernel averages 379 us over 20 launches from idle and
    294 us in steady state), so every timed region starts at steady state.  The iteration count
    comes from a short probe and is agreed over the ranks (max), so steps that contain collectives
    stay matched."""
    seconds = SPINUP_S if seconds is None else seconds
    if seconds <= 0:
        return
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    n = int(seconds / max((time.perf_counter() - t0) / 3, 1e-6)) + 1
    if world > 1:
        t = torch.tensor([n], dtype=torch.int64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        n = int(t.item())
    for i in range(n):
        fn()
        if i % 8 == 7:
            torch.cuda.synchronize()


def timed(fn, steps, warmup, world, tail=None):
    """Spin-up, W untimed warmup steps, then exactly K steps between barrier+synchronize; returns
    (max-over-ranks wall seconds, mean device ms per step from two HIP events on the launch stream
    around the K steps -- no markers between steps, which would themselves open dispatch gaps).
    ``tail``: a step that leaves work for the next one (the cross-step C5 exchange) is completed by
    it -- once before the timed region (the warmup's leftover) and once inside it, after the K
    steps, so the region holds exactly K steps' work."""
    spinup(fn, world=world)
    for _ in range(warmup):
        fn()
    if tail is not None:
        tail()
    sync_all(world)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(steps):
        fn()
    if tail is not None:
        tail()
    e1.record()
    sync_all(world)
    wall = time.perf_counter() - t0
    dev_ms = e0.elapsed_time(e1) / steps
    if world > 1:
        t = torch.tensor([wall], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    return wall, dev_ms


def kernel_ms(fn, reps=50, warmup=2):
    """Mean device time of one launch of ``fn`` (HIP events on torch's current stream, which is the
    stream every gr_amd op enqueues on), after a short spin-up (clock ramp)."""
    spinup(fn, min(SPINUP_S, 0.3))
    for _ in range(warmup):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


# one gr_score_topk_f32 call: the tile pass (MODE 2: 32-row tile maxima,
# at 1M rows; MODE 3: 16-row half tiles, topk_half's choice on a shard) + the select kernel
TOPK_PASS = "score_topk_kernel<128,10,2>"
TOPK_PASS_HALF = "score_topk_kernel<128,10,3>"
TOPK_CALL_KERNELS = [TOPK_PASS, TOPK_PASS_HALF, "topk_select_kernel<128,10>"]


def call_traffic(leg, kernels, anchor):
    """HBM bytes per call from the committed PMC summary (profiles/traffic.json, written per bench
    leg and launch shape by scripts/pmc_traffic.py): the bytes of every launch in ``leg`` whose
    kernel name starts with one of ``kernels``, divided by the number of launches of ``anchor``
    (one per call).  None when the leg was not profiled."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None, None
    t = json.load(open(p))
    groups = t.get("legs", {}).get(leg)
    if not groups:
        return None, None
    name = lambda key: key.rsplit("@", 1)[0]
    calls = sum(g["launches"] for k, g in groups.items() if name(k).startswith(anchor))
    if calls == 0:
        return None, None
    tot = sum(g["bytes_per_launch"] * g["launches"] for k, g in groups.items()
              if any(name(k).startswith(p) for p in kernels))
    return tot / calls, f"{t.get('source', '')}, leg {leg}"


# the rocprofv3 --kernel-trace summary of the default bench command on this tree
# (scripts/trace_stats.py over the same run as profiles/r06/rocprof_kernel_stats.csv)
ROCPROF_TRACE = os.path.join("profiles", "r06", "rocprof_trace_stats.csv")


def rocprof_median_us(kernel, near_ms):
    """Median launch duration (us) of ``kernel`` (prefix of the demangled name, spaces ignored) in the
    committed rocprofv3 trace summary, so the bench line carries the profiler's figure beside its own
    event timing.  A kernel profiled at several launch shapes (C2 / C4 encoders,
    the C5 / shard top-k passes) is matched to the shape whose median is nearest ``near_ms``; the
    chosen shape's grid is reported.  None when the summary is absent."""
    import csv
    p = os.path.join(ROOT, ROCPROF_TRACE)
    if not os.path.exists(p):
        return None
    rows = []
    for r in csv.DictReader(open(p)):
        name = r.get("kernel", "").replace("void ", "").replace("gr::", "").replace(" ", "")
        if name.startswith(kernel.replace(" ", "")):
            rows.append((float(r["median_us"]), int(r["grid_threads"]), int(r["calls"])))
    if not rows:
        return None
    med, grid, calls = min(rows, key=lambda x: abs(x[0] - near_ms * 1e3))
    return {"median_us": med, "grid_threads": grid, "launches": calls, "shapes_profiled": len(rows)}


def roofline(kernel, flop, ms, leg, bound="mfma", call_kernels=None, note=None):
    """``kernel`` names the dominant kernel (prefix of its profiled name); ``call_kernels`` lists
    the kernel-name prefixes one timed call launches (default: ``kernel`` alone), so ``traffic``
    is per call, like ``achieved``.  ``frac`` is from this run's HIP-event timing; ``frac_rocprof``
    from the committed rocprofv3 median of the same kernel (``rocprof_source``)."""
    ach = flop / (ms * 1e-3) / 1e12
    tr, src = call_traffic(leg, call_kernels or [kernel], kernel)
    rp = rocprof_median_us(kernel, ms) if not call_kernels or call_kernels == [kernel] else None
    extra = {}
    if rp is not None:
        extra = {"kernel_us_rocprof_median": rp["median_us"],
                 "frac_rocprof": flop / (rp["median_us"] * 1e-6) / 1e12 / FP32_PEAK_TFLOPS,
                 "rocprof_source": f"{ROCPROF_TRACE} (grid {rp['grid_threads']}, {rp['launches']} launches)"}
    return {"bound": bound, "achieved": ach, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": ach / FP32_PEAK_TFLOPS, **extra, "traffic": tr, "traffic_source": src, "kernel": kernel,
            "flop_per_launch": flop, "kernel_ms": ms, **({"note": note} if note else {})}


def cpu_threads():
    n = len(os.sched_getaffinity(0))
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", n))))


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_median(fn, units, unit, sample, warm=3, reps=10, agree=None):
    """the CPU restatement timed with 3 warmups then the median of 10 calls, on
    ``cpu_threads()`` host threads; returns the cpu_baseline object (``units`` per call).
    ``agree(out)`` compares the last call's output with the GPU's on the same inputs; its dict is
    reported as ``agreement`` (§8(d): the restatement's agreement on the bench host, reported
    separately from the fixture-host parity)."""
    torch.set_num_threads(cpu_threads())
    for _ in range(warm):
        fn()
    ts = []
    out = None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    med = float(np.median(ts))
    res = {"value": units / med, "unit": unit, "cores": torch.get_num_threads(), "kind": "port",
           "cpu": cpu_model(), "timing": f"{warm} warmups + median of {reps} calls "
           f"(median {med * 1e3:.1f} ms, min {min(ts) * 1e3:.1f}, max {max(ts) * 1e3:.1f})", "sample": sample}
    if agree is not None:
        res["agreement"] = agree(out)
    return res


def rq_agreement(cpu_idx, gpu_idx, detail=None):
    """Rows whose semantic IDs differ between the host restatement and the GPU, each characterised
    against the near-tie certificate: ``detail`` = (GPU best [n, L], GPU gap
    [n, L], GPU z [n, e], host z [n, e]).  A differing row is "flagged" when some level's GPU
    best/second-best gap is within ``near_tie_bound`` (gr_amd.rqvae: the fp32 disagreement two
    implementations whose encoder outputs differ by |dz| <= Z_TAU |z| can show); an unflagged
    differing row would be a real parity break.  Also reported: this host's encoder deviation
    max |z_host - z_gpu| / |z_gpu| against Z_TAU, the assumption the certificate rests on."""
    from gr_amd.rqvae import Z_TAU, near_tie_bound
    cpu_idx, gpu_idx = cpu_idx.cpu(), gpu_idx.cpu()
    diff = (cpu_idx != gpu_idx).any(1)
    res = {"rows": int(cpu_idx.shape[0]), "rows_ids_differ": int(diff.sum()),
           "note": "oracle/rq_oracle (torch CPU ops, this host's MKL) vs the GPU get_indices on the same "
                   "items; the bit-exact claim is pinned on the fixture host's reference outputs "
                   "(tests/golden), this count is this host's CPU path"}
    if detail is None:
        return res
    best, gap, zg, zc = (t.detach().cpu().double() for t in detail)
    zn2 = (zg * zg).sum(1)
    bound = near_tie_bound(best, gap, zn2)
    flagged = (gap <= bound).any(1)
    dzr = (zc - zg).norm(dim=1) / zn2.sqrt().clamp_min(1e-30)
    rows = []
    for r in torch.nonzero(diff).flatten().tolist()[:32]:
        lv = int(torch.nonzero(cpu_idx[r] != gpu_idx[r]).flatten()[0])
        rows.append({"row": r, "first_level_differing": lv, "gpu_gap": float(gap[r, lv]),
                     "near_tie_bound": float(bound[r, lv]), "gap_over_bound": float(gap[r, lv] / bound[r, lv]),
                     "flagged": bool(flagged[r]), "host_dz_over_z": float(dzr[r]),
                     "host_z_bitwise_equal": bool(torch.equal(zc[r], zg[r]))})
    res.update({"rows_ids_differ_flagged": int((diff & flagged).sum()),
                "rows_ids_differ_unflagged": int((diff & ~flagged).sum()),
                "rows_flagged_total": int(flagged.sum()),
                "host_z_rows_bitwise_equal": int((zc == zg).all(1).sum()),
                "host_dz_over_z_max": float(dzr.max()), "z_tau": Z_TAU,
                "host_dz_within_z_tau": bool(float(dzr.max()) <= Z_TAU),
                "differing_rows": rows,
                "certificate": "flagged = some level's GPU best/second-best distance gap <= near_tie_bound "
                               "(gr_amd/rqvae.py): an fp32 tie window two implementations with |dz| <= "
                               "Z_TAU |z| may resolve either way"})
    return res


def sas_agreement(cpu_logits, gpu_logits, seed=0):
    """Max row-scaled logit error and strict ranks (SASRec/evaluate.py:27-32, column 0 masked) on
    the same users, with half the targets from the host path's top-20 and half uniform."""
    c = cpu_logits.float()
    g_ = gpu_logits.float().cpu()
    scale = c.abs().amax(1)
    err = float(((g_ - c).abs().amax(1) / scale).max())
    B, rows = c.shape
    rng = np.random.default_rng(seed)
    cm, gm = c.clone(), g_.clone()
    cm[:, 0] = -1e9
    gm[:, 0] = -1e9
    top20 = torch.topk(cm, 20, dim=1).indices.numpy()
    tg = torch.from_numpy(np.where(rng.random(B) < 0.5, top20[np.arange(B), rng.integers(0, 20, B)],
                                   rng.integers(1, rows, B)).astype(np.int64))[:, None]
    rc = (cm > cm.gather(1, tg)).sum(1) + 1
    rg = (gm > gm.gather(1, tg)).sum(1) + 1
    return {"users": B, "max_row_scaled_logit_err": err, "tolerance": 1e-5,
            "ranks_differ": int((rc != rg).sum()), "hr10_cpu": float((rc <= 10).double().mean()),
            "hr10_gpu": float((rg <= 10).double().mean()),
            "note": "oracle/sasrec_oracle.predict on this host's CPU vs the GPU's logits of the same users; "
                    "targets half from the host path's top-20, half uniform"}


def cpu_rq_baseline(model, n_items, tag):
    """Oracle restatement of get_indices (oracle/rq_oracle.py) on host cores, one call of
    ``n_items`` synthetic items of the same workload; ``agreement``: its IDs against the GPU's."""
    from oracle import rq_oracle
    lin = model.encoder.linears()
    ws = [l.weight.detach().cpu() for l in lin]
    bs = [l.bias.detach().cpu() for l in lin]
    cbs = [c.cpu() for c in model.rq.codebooks()]
    xg = synth.items(n_items, 12345, "cuda")
    gpu_idx = model.get_indices(xg).cpu()
    _, best, gap, zg = ops.rq_encode(xg, binding=model.encode_binding(), with_gap=True, with_z=True)
    x = xg.cpu()
    torch.set_num_threads(cpu_threads())
    zc = rq_oracle.mlp_encode(x, ws, bs)   # this host's encoder output for the same call (one batch)
    return cpu_median(lambda: rq_oracle.get_indices(x, ws, bs, cbs), n_items, "items/s",
                      f"oracle/rq_oracle.get_indices, {tag}: batch of {n_items} synthetic items (fp32 torch CPU)",
                      agree=lambda out: rq_agreement(out, gpu_idx, (best, gap, zg, zc)))


def cpu_sas_baseline(model, B, n, items, tag, table=None, params=None):
    """Oracle restatement of predict (oracle/sasrec_oracle.py) on host cores, one call of B users
    (``table``: the full [items+1, d] item table when the model holds a compact one; the GPU side
    then rebuilds the compact model for these users from ``params``); ``agreement``: its logits and
    ranks against the GPU's on the same users."""
    from oracle import sasrec_oracle
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    seqs_g = synth.sequences(B, n, items, 777, "cuda")
    if table is not None:
        sd["item_emb.weight"] = table.detach().cpu()
        mr, sr = synth.sasrec_rank_model(items, params, seqs_g, seqs_g.device, seed=5)
        gpu_logits = ops.score(mr.last_hidden(sr), table).cpu()
        del mr
    else:
        gpu_logits = model.predict(seqs_g).cpu()
    seqs = seqs_g.cpu()
    return cpu_median(lambda: sasrec_oracle.predict(seqs, sd, model.num_blocks, model.num_heads, 1e-8),
                      B, "seqs/s", f"oracle/sasrec_oracle.predict, {tag}: batch of {B} users "
                      f"(d {model.d}, n {n}, {items}-item catalog, logits [B, {items + 1}])",
                      agree=lambda out: sas_agreement(out, gpu_logits))


def bench_rq_c2(a, world, rank, dev):
    L, K = 3, 256
    model = synth.rqvae_model(L, K, dev)
    x = synth.items(a.rq_items, 1000 + rank, dev)
    wall, dev_ms = timed(lambda: model.get_indices(x), a.steps, a.warmup, world)
    # the encoder's share of the call = the call minus the quantize kernel timed alone on the same
    # z (ops.rq_mlp would also time the per-call weight pack that get_indices caches)
    z = model.encoder(x)
    cbs = model.rq.codebooks()
    quant_ms = kernel_ms(lambda: ops.rq_quantize(z, cbs))
    enc_ms = dev_ms - quant_ms
    line = {
        "metric": METRIC, "value": a.rq_items * world * a.steps / wall, "unit": "items/s",
        "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": wall / a.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": "rq_c2: RQ-VAE get_indices, 3x256 codebooks, in 768 -> [256,128] -> "
                               "e 32, data-derived codebooks, BERT-statistics item embeddings",
                   "items_per_rank_per_step": a.rq_items, "global_batch": a.rq_items * world,
                   "parallelism": f"item-sharded x{world}, no collective"},
        "roofline": roofline("rq_encoder_kernel<256,128>", ENC_FLOP_PER_ITEM * a.rq_items, enc_ms, "c2",
                             call_kernels=["rq_encoder_kernel", "rq_leftover_kernel"],
                             note="the encoder launches of one call (rq_encoder_kernel, plus rq_leftover_kernel for "
                                  "the leftover tiles' layers 2-3): the call's device time minus the quantize "
                                  "kernel timed alone"),
        "call": {"kernels": "rq_encoder_kernel + rq_leftover_kernel + rq_quantize_kernel", "device_ms": dev_ms,
                 "device_ms_per_rank": per_rank(dev_ms, world),
                 "flop_per_item": rq_flop_per_item(L, K),
                 "frac_of_fp32_peak": rq_flop_per_item(L, K) * a.rq_items / (dev_ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS,
                 "hbm_algorithmic_GBs": rq_bytes_per_item(L) * a.rq_items / (dev_ms * 1e-3) / 1e9,
                 "quantize_ms": quant_ms},
    }
    return line, model


def bench_rq_c4(a, world, rank, dev):
    """C4: a fixed catalog of c4_items split over the ranks (strong scaling), 4x1024 codebooks."""
    L, K = 4, 1024
    model = synth.rqvae_model(L, K, dev, seed=4)
    lo = a.c4_items * rank // world
    hi = a.c4_items * (rank + 1) // world
    x = synth.items(hi - lo, 4000 + rank, dev)
    steps, warm = max(2, min(a.steps, 5)), 1
    wall, dev_ms = timed(lambda: model.get_indices(x), steps, warm, world)
    enc_ms = kernel_ms(lambda: ops.rq_encode(x, binding=model.encode_binding()), reps=3)
    res = {"metric": "items_encoded/s", "value": a.c4_items * steps / wall, "unit": "items/s",
            "scaling": "strong", "ms_per_step": wall / steps * 1e3, "steps": steps,
            "config": {"workload": "rq_c4: RQ-VAE get_indices, 4x1024 codebooks, in 768 -> [256,128] -> e 32",
                       "catalog_items": a.c4_items, "items_per_rank": hi - lo,
                       "parallelism": f"item-sharded x{world}, no collective"},
            "call": {"device_ms": dev_ms, "device_ms_per_rank": per_rank(dev_ms, world),
                     "flop_per_item": rq_flop_per_item(L, K),
                     "frac_of_fp32_peak": rq_flop_per_item(L, K) * (hi - lo) / (dev_ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS,
                     "encode_call_ms_50rep_mean": enc_ms}}
    return res, model


def bench_sas_c3(a, world, rank, dev):
    d, n, items = 64, 50, 100_000
    p = synth.sasrec_params(d, n, 2, 1, 64, dev)
    model = synth.sasrec_model(items, p, dev)
    seqs = synth.sequences(a.sas_batch, n, items, 2000 + rank, dev)
    # timed through the drop-in surface: model.predict(seqs) allocates its fresh contiguous [B, N+1]
    # logits every call (the reference's matmul layout, model.py:107), as evaluate.py:26 sees it
    assert model.contiguous_logits
    wall, dev_ms = timed(lambda: model.predict(seqs), a.steps, a.warmup, world)
    out = torch.empty((a.sas_batch, items + 1), dtype=torch.float32, device=dev)   # predict's layout
    h = model.last_hidden(seqs)
    table = model.item_emb.weight.detach()
    score_ms = kernel_ms(lambda: ops.score(h, table, out=out))
    fwd_ms = kernel_ms(lambda: model.last_hidden(seqs))
    targets = torch.randint(1, items + 1, (a.sas_batch,), generator=torch.Generator(device=dev).manual_seed(5), device=dev)
    rank_ms = kernel_ms(lambda: ops.score_rank(h, table, targets))
    fl = sas_flop_per_user(d, n, items)
    th = True   # the fused kernel's final block runs in the H form
    fl_exe = sas_exec_flop_per_user(d, n, items, causal=False, tail_h=th)
    fwd_exe = sas_exec_flop_per_user(d, n, -1, causal=False, tail_h=th)
    res = {"metric": "seqs_scored/s", "value": a.sas_batch * world * a.steps / wall, "unit": "seqs/s",
           "ms_per_step": wall / a.steps * 1e3, "scaling": "weak",
           "config": {"workload": "sas_c3: SASRec predict, 2 blocks, d 64, n 50, H 1, mlp 64, "
                                  "100k-item full-catalog logits written", "users_per_rank_per_step": a.sas_batch,
                      "parallelism": f"user-sharded x{world}, no collective"},
           "roofline": roofline("score_rot_kernel<64" if a.sas_batch * (items + 1) * 4 > 160e6 else "score_direct_kernel<64",
                                2 * d * (items + 1) * a.sas_batch, score_ms, "sasrec"),
           "call": {"device_ms": dev_ms, "device_ms_per_rank": per_rank(dev_ms, world), "flop_per_user": fl,
                    "frac_of_fp32_peak": fl * a.sas_batch / (dev_ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS,
                    "flop_per_user_executed": fl_exe,
                    "frac_of_fp32_peak_executed": fl_exe * a.sas_batch / (dev_ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS,
                    "forward_ms": fwd_ms, "forward_flop_per_user_executed": fwd_exe,
                    "forward_frac_executed": fwd_exe * a.sas_batch / (fwd_ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS,
                    "executed_note": "block 0 in full (the one-wave kernel computes the whole n x n "
                                     "attention tile), the last block at position n-1 only (H form: "
                                     "W_k^T q, the n LayerNorm rows dotted twice, W_v u; no K|V of the "
                                     "n tokens)" if th else
                                     "block 0 in full (the one-wave kernel computes the whole n x n "
                                     "attention tile), the last block's K|V for all n tokens and the "
                                     "rest at position n-1 only",
                    "score_ms": score_ms,
                    "logits_write_GBs": a.sas_batch * (items + 1) * 4 / (score_ms * 1e-3) / 1e9},
           "rank_fused": {"note": "forward + target logit + strict count, logits never written",
                          "value": a.sas_batch / ((fwd_ms + rank_ms) * 1e-3), "unit": "seqs/s",
                          "rank_ms": rank_ms,
                          "frac_of_fp32_peak": 2 * d * (items + 1) * a.sas_batch / (rank_ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS}}
    return res, model, (n, items)


def bench_sas_c5(a, world, rank, dev, time_it=True):
    """C5: the catalog sharded over the ranks; every rank runs the transformer for its share of the
    users, hidden states are all-gathered, each rank scores ALL users against its catalog shard,
    then counts are all-reduced and top-10 lists all-gathered (gr_amd.dist)."""
    from gr_amd import dist as D
    d, n, items, B = 128, 200, a.c5_items, a.c5_batch * world   # c5_batch users per rank (weak)
    p = synth.sasrec_params(d, n, 2, 1, 64, dev)
    seqs = synth.sequences(B, n, items, 5000, dev)            # same users on every rank
    targets = torch.randint(1, items + 1, (B,), generator=torch.Generator(device=dev).manual_seed(6), device=dev)
    ulo, uhi = D.shard_range(B, rank, world)
    usizes = [D.shard_range(B, r_, world)[1] - D.shard_range(B, r_, world)[0] for r_ in range(world)]
    lo, hi = D.shard_range(items + 1, rank, world)
    # each rank builds only its catalog shard (scored) and the rows its own users' histories gather
    # (forward), both from the position-keyed synth.table_rows: every world size scores the same table
    t0 = time.perf_counter()
    shard = synth.table_rows(torch.arange(lo, hi, device=dev), d, 7, dev)
    model, lseqs = synth.sasrec_rank_model(items, p, seqs[ulo:uhi], dev, seed=5)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t0

    def gather_h():
        hl = model.last_hidden(lseqs)
        return D.all_gather_rows(hl, sizes=usizes) if dist.is_initialized() else hl

    pipe = D.ShardedRankPipeline(shard, lo, k=10)

    def make_step(mode):
        """(step, tail) of one exchange form: "serial" (dist.sharded_rank_topk), "split" (the step's
        users cut into --c5-pipeline sub-batches, each one's exchange under the next one's scoring:
        dist.sharded_rank_topk_batches), "xstep" (the whole batch scored at once, its exchange under
        the NEXT step's forward + all-gather: dist.ShardedRankPipeline)."""
        P = max(2, a.c5_pipeline)
        cuts = [B * j // P for j in range(P + 1)]

        def serial():
            return D.sharded_rank_topk(gather_h(), shard, lo, targets, k=10)

        def split():
            h = gather_h()
            r = D.sharded_rank_topk_batches([h[x:y] for x, y in zip(cuts[:-1], cuts[1:])], shard, lo,
                                            [targets[x:y] for x, y in zip(cuts[:-1], cuts[1:])], k=10)
            return tuple(torch.cat(t) for t in zip(*r))

        def xstep():
            return pipe.submit(gather_h(), targets)
        return {"serial": (serial, None), "split": (split, None), "xstep": (xstep, pipe.flush)}[mode]

    if not time_it:   # setup only (the shard leg alone): no C5 launches in its profile
        return None, model, gather_h(), targets, shard
    steps, warm = max(2, min(a.steps, 10)), 2
    # the exchange form: --c5-exchange, or ("auto", the default) at N > 1 each form is timed on a
    # few steps, max over ranks (so every rank picks the same), and the fastest runs; at N = 1
    # there is no exchange to hide ("serial": a single shard, no collectives at all)
    probe = None
    if a.c5_exchange != "auto":
        mode = a.c5_exchange
    elif not dist.is_initialized():
        mode = "serial"
    else:
        probe = {}
        for mc in C5_EXCHANGES:
            st_, tl_ = make_step(mc)
            pw, _ = timed(st_, 3, 1, world, tail=tl_)
            probe[f"{mc}_ms_per_step"] = pw / 3 * 1e3
        mode = min(C5_EXCHANGES, key=lambda x: probe[f"{x}_ms_per_step"])
    step, tail = make_step(mode)
    wall, dev_ms = timed(step, steps, warm, world, tail=tail)
    r = step()
    if tail is not None:
        r = tail()
    check = result_checksum(r, world)
    h = gather_h()
    ts = torch.zeros(B, device=dev)
    topk_ms = kernel_ms(lambda: ops.score_topk(h, shard, 10, lo, thresholds=ts, mask_col0=(lo == 0)))
    fwd_ms = kernel_ms(lambda: model.last_hidden(lseqs))
    fl_ref = sas_flop_per_user(d, n, items)
    th = True   # the C5 forward's final block runs in the H form (sas_tail_h2_kernel)
    fl_exe = sas_exec_flop_per_user(d, n, items, causal=True, tail_h=th)
    fwd_exe = sas_exec_flop_per_user(d, n, -1, causal=True, tail_h=th)
    res = {"metric": "seqs_scored/s", "value": B * steps / wall, "unit": "seqs/s", "scaling": "weak",
            "ms_per_step": wall / steps * 1e3, "steps": steps,
            "config": {"workload": "sas_c5: SASRec d 128, n 200, 2 blocks, 1M-item catalog, rank + top-10",
                       "users_per_step": B, "users_per_rank": a.c5_batch, "catalog_rows": items + 1,
                       "rows_per_rank": hi - lo,
                       "users_forwarded_per_rank": uhi - ulo, "table_rows_built_per_rank": (hi - lo) + model.item_num,
                       "setup_s": setup_s,
                       "exchange": mode, "exchange_probe": probe,
                       "pipeline_sub_batches": max(2, a.c5_pipeline) if mode == "split" else 1,
                       "parallelism": f"catalog-sharded x{world}: RCCL all-gather h + top-k, all-reduce counts, "
                       f"{mode} exchange" if world > 1 else "single shard"},
            "result_checksum": check,
            "roofline": roofline(TOPK_PASS, 2 * d * (hi - lo) * B, topk_ms, "c5",
                                 call_kernels=TOPK_CALL_KERNELS,
                                 note="one gr_score_topk_f32 call: the tile pass (scores, strict counts, "
                                      "per-user 32-row tile maxima) + the select kernel (re-scores the tiles "
                                      "at or above the k-th tile max); flop counts the scoring GEMM once; "
                                      "traffic is the whole call's"),
            "call": {"device_ms_rank0": dev_ms, "device_ms_per_rank": per_rank(dev_ms, world),
                     "flop_per_user": fl_ref, "flop_per_user_executed": fl_exe,
                     "frac_of_fp32_peak": fl_ref * B / world / (wall / steps) / 1e12 / FP32_PEAK_TFLOPS,
                     "frac_of_fp32_peak_executed": fl_exe * B / world / (wall / steps) / 1e12 / FP32_PEAK_TFLOPS,
                     "forward_ms": fwd_ms, "forward_flop_per_user_executed": fwd_exe,
                     "forward_frac_executed": fwd_exe * (uhi - ulo) / (fwd_ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS,
                     "score_topk_ms": topk_ms,
                     "note": "rank + top-10 fused into the scoring pass (gr_score_topk_f32): the "
                             "[B, rows] logits are never written; 'executed' counts causal attention "
                             "(n(n+1)/2 query-key pairs) and the final block at position n-1 only, as "
                             "the kernels run it; frac from the max-over-ranks wall time per step"}}
    return res, model, h, targets, shard


def sas_train_bytes(B, n, d, rows, J):
    """Algorithmic HBM bytes of one training-side scoring step (forward + backward of
    gr_sampled_bce_*): every operand read or written once (features twice: forward and backward),
    the gathered table rows once per pass, the dense dM written once plus a read-modify-write of
    the touched rows."""
    P = B * n
    fwd = P * d * 4 + (P + B * J) * d * 4 + P * 8 + B * J * 8 + P * (J + 2) * 4
    bwd = 2 * P * d * 4 + P * (J + 1) * 4 + (P + B * J) * d * 4 + P * d * 4 + rows * d * 4 \
        + 2 * (P + B * J) * d * 4
    return fwd + bwd


def bench_sas_train(a, world, rank, dev):
    """the training-side scoring of SASRec/train.py:131-167 at C3 shapes with the
    reference's training batch (main.py: batch_size 128, num_neg_samples 10, loss_eps 1e-24):
    forward + backward of ops.sampled_bce_loss (no [B, n, N+1] score matrix), user-sharded."""
    B, n, d, items, J = a.train_batch, 50, 64, 100_000, 10
    g = torch.Generator(device=dev).manual_seed(3000 + rank)
    feats = (0.3 * torch.randn(B, n, d, generator=g, device=dev)).requires_grad_(True)
    table = (0.3 * torch.randn(items + 1, d, generator=g, device=dev)).requires_grad_(True)
    lens = torch.randint(3, n + 1, (B,), generator=g, device=dev)
    targets = torch.randint(1, items + 1, (B, n), generator=g, device=dev)
    targets[torch.arange(n, device=dev)[None, :] < (n - lens)[:, None]] = 0
    inputs = torch.roll(targets, 1, dims=1)          # s_t = o_{t-1}, the train-mode pairs
    inputs[:, 0] = 0
    negs = ops.neg_samples(inputs, items, J)

    def step():   # train.py:142 (negatives) + 134-167 (scores, loss, backward); the transformer is the caller's
        ng = ops.neg_samples(inputs, items, J)
        bl, valid = ops.sampled_bce_loss(feats, table, targets, ng, 1e-24)
        feats.grad = table.grad = None
        (bl / valid).backward()

    def dense_step():   # train.py:134-167 as written, in torch on the same GPU (rocBLAS GEMMs)
        sm = torch.matmul(feats, table.t())
        mask = (targets != 0).float()
        ne = negs.unsqueeze(1).expand(-1, n, -1)
        ps = torch.gather(sm, 2, targets.unsqueeze(-1)).squeeze(-1)
        ns = torch.gather(sm, 2, ne)
        pl = -torch.log(torch.sigmoid(ps) + 1e-24) * mask
        nl = (-torch.log(1 - torch.sigmoid(ns) + 1e-24) * mask.unsqueeze(-1)).sum(-1)
        feats.grad = table.grad = None
        ((pl + nl).sum() / mask.sum()).backward()

    eager_wall, eager_dev_ms = timed(step, a.steps, a.warmup, world)
    # the same step captured once and replayed (ops.SasTrainStepGraph: one graph launch per step,
    # fresh device-seeded negatives each replay) -- the leg's value
    feats.grad = table.grad = None
    gstep = ops.SasTrainStepGraph(feats, table, inputs, targets, items, J, 1e-24, seed=3000 + rank)
    wall, dev_ms = timed(gstep.replay, a.steps, a.warmup, world)
    dense_ms = kernel_ms(dense_step, reps=10)
    nbytes = sas_train_bytes(B, n, d, items + 1, J)
    tr, tr_src = call_traffic("train", ["neg_sample_kernel", "bce_"], "neg_sample_kernel")
    res = {"metric": "train_seqs_scored/s", "value": B * world * a.steps / wall, "unit": "seqs/s",
           "ms_per_step": wall / a.steps * 1e3, "scaling": "weak",
           "config": {"workload": f"sas_train: SASRec train.py:131-167 scoring + sampled BCE, forward + "
                                  f"backward, B {B}, n {n}, d {d}, {items}-item table, {J} negatives; "
                                  f"the step captured as one graph (ops.SasTrainStepGraph)",
                      "users_per_rank_per_step": B, "parallelism": f"user-sharded x{world}, no collective"},
           "eager": {"note": "the same step issued op by op from Python (host-launch bound)",
                     "value": B * world * a.steps / eager_wall, "ms_per_step": eager_wall / a.steps * 1e3,
                     "step_device_ms": eager_dev_ms},
           "roofline": {"bound": "hbm", "achieved": nbytes / (dev_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": nbytes / (dev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                        "traffic": tr, "traffic_source": tr_src and tr_src + " (the gr:: kernels of the "
                                                                    "step as profiled)",
                        "kernel": "whole step (gr_neg_samples + gr_sampled_bce fwd + bwd + the dM fill kernel)",
                        "bytes_per_step": nbytes, "step_device_ms": dev_ms},
           "reference_formulation_gpu": {"note": "train.py:134-167 as written ([B, n, N+1] score matrix, "
                                                 "gathers, dense backward) in torch on the same GPU, "
                                                 "negatives precomputed (the reference draws them on the host)",
                                         "ms_per_step": dense_ms, "speedup": dense_ms / dev_ms}}
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle import sasrec_oracle
        f, w, t, si = feats.detach().cpu(), table.detach().cpu(), targets.cpu(), inputs.cpu().numpy()
        rng = np.random.RandomState(0)

        def cpu_step():
            ng = sasrec_oracle.neg_samples(si, items, J, rng)
            sasrec_oracle.train_loss_grads(f, w, t, ng, 1e-24)
        res["cpu_baseline"] = cpu_median(cpu_step, B, "seqs/s",
                                         f"oracle get_neg_samples (train.py:15-30, numpy) + train_loss_grads "
                                         f"(train.py:134-167, torch CPU), one step of B {B}")
    return res


def sas_step_flop_per_user(d, n, mlp=64, blocks=2, J=10):
    """One training step of SASRec/train.py:131-173 per user at the reference formulation's
    transformer (sas_flop_per_user without the catalog scoring) x 3 (forward + backward), plus the
    sampled scoring's 2 * n * (1 + J) * d per pass (forward, and the backward's two products)."""
    fwd = sas_flop_per_user(d, n, 0, mlp, blocks) - 2 * d
    return 3 * fwd + 3 * 2 * n * (1 + J) * d


def bench_sas_train_step(a, world, rank, dev):
    """SURVEY §8(f) row 4, the whole SASRec training step (SASRec/train.py:131-173) at the
    reference's training batch (main.py: batch 128, dropout 0.2, Adam lr 1e-3 betas (0.9, 0.98),
    10 negatives) on C3 shapes (d 64, n 50, 100k items): the transformer forward + backward on the
    fused training kernels (dropout on), GPU negatives, the fused sampled BCE, the weight-gradient
    GEMMs and the Adam step, captured as one graph (ops.SasTrainGraph) -- next to the same step
    issued eagerly, the same captured step with the transformer under torch autograd
    (module by module, SASRec.fused_train = False), and the reference's own formulation
    ([B, n, N+1] score matrix, torch modules) eagerly on the same GPU."""
    B, n, d, items, J = a.train_batch, 50, 64, 100_000, 10
    prm = synth.sasrec_params(d, n, 2, 1, 64, dev)
    g = torch.Generator(device=dev).manual_seed(4000 + rank)
    lens = torch.randint(3, n + 1, (B,), generator=g, device=dev)
    targets = torch.randint(1, items + 1, (B, n), generator=g, device=dev)
    targets[torch.arange(n, device=dev)[None, :] < (n - lens)[:, None]] = 0
    inputs = torch.roll(targets, 1, dims=1)
    inputs[:, 0] = 0

    def make(capturable, fused=True):
        m = synth.sasrec_model(items, prm, dev, seed=11).train()   # dropout 0.2 (main.py)
        m.fused_train = fused
        # Adam(lr 1e-3, betas (0.9, 0.98)) as train.py:107; the fused multi-tensor implementation
        # (same update) for the kernel path -- the foreach one costs ~70 small launches per step
        return m, torch.optim.Adam(m.parameters(), lr=1e-3, betas=(0.9, 0.98), capturable=capturable,
                                   fused=fused or None)

    m1, o1 = make(True)
    gstep = ops.SasTrainGraph(m1, o1, inputs, targets, items, J, 1e-24, seed=5000 + rank)
    wall, dev_ms = timed(gstep.replay, a.steps, a.warmup, world)
    del gstep, m1, o1
    m2, o2 = make(False)

    def eager():   # the same step op by op
        o2.zero_grad()
        h = m2(inputs)
        ng = ops.neg_samples(inputs, items, J)
        bl, valid = ops.sampled_bce_loss(h, m2.item_emb.weight, targets, ng, 1e-24)
        (bl / valid.clamp(min=1.0)).backward()
        o2.step()
    e_wall, _ = timed(eager, a.steps, a.warmup, world)
    m4, o4 = make(True, fused=False)
    mstep = ops.SasTrainGraph(m4, o4, inputs, targets, items, J, 1e-24, seed=6000 + rank)
    ma_ms = kernel_ms(mstep.replay, reps=20)
    del mstep, m4, o4
    m3, o3 = make(False, fused=False)
    negs = ops.neg_samples(inputs, items, J)

    def reference():   # train.py:131-173 as written (score matrix, torch modules), negatives precomputed
        o3.zero_grad()
        h = m3(inputs)
        sm = torch.matmul(h, m3.item_emb.weight.t())
        mask = (targets != 0).float()
        ps = torch.gather(sm, 2, targets.unsqueeze(-1)).squeeze(-1)
        ns = torch.gather(sm, 2, negs.unsqueeze(1).expand(-1, n, -1))
        pl = -torch.log(torch.sigmoid(ps) + 1e-24) * mask
        nl = (-torch.log(1 - torch.sigmoid(ns) + 1e-24) * mask.unsqueeze(-1)).sum(-1)
        ((pl + nl).sum() / mask.sum()).backward()
        o3.step()
    r_ms = kernel_ms(reference, reps=10)
    fl = sas_step_flop_per_user(d, n, 64, 2, J) * B
    step_ms = wall / a.steps * 1e3
    res = {"metric": "train_steps_seqs/s", "value": B * world * a.steps / wall, "unit": "seqs/s",
           "ms_per_step": step_ms, "scaling": "weak",
           "config": {"workload": f"sas_train_step: SASRec train.py:131-173 whole step (transformer forward "
                                  f"+ backward with dropout 0.2 on the fused training kernels, {J} GPU negatives, "
                                  f"fused sampled BCE, weight-gradient GEMMs, Adam), B {B}, n {n}, d {d}, "
                                  f"{items}-item table, one captured graph",
                      "users_per_rank_per_step": B, "parallelism": f"user-sharded x{world} (data parallel "
                                                                   f"without the gradient all-reduce)"},
           "roofline": {"bound": "mfma", "achieved": fl / (dev_ms * 1e-3) / 1e12, "peak": FP32_PEAK_TFLOPS,
                        "unit": "TFLOP/s", "frac": fl / (dev_ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS,
                        "traffic": None, "kernel": "whole step (latency-bound: 128 one-sequence workgroups)",
                        "flop_per_step": fl, "step_device_ms": dev_ms},
           "eager": {"note": "the same step issued op by op", "value": B * world * a.steps / e_wall,
                     "ms_per_step": e_wall / a.steps * 1e3},
           "captured_module_autograd": {"note": "the same captured step with the transformer under torch "
                                                "autograd, module by module (SASRec.fused_train = False)",
                                        "ms_per_step": ma_ms, "speedup": ma_ms / step_ms},
           "reference_formulation_gpu": {"note": "train.py:131-173 as written ([B, n, N+1] score matrix, torch "
                                                 "modules) on the same GPU, negatives precomputed (the reference "
                                                 "draws them on the host)",
                                         "ms_per_step": r_ms, "speedup": r_ms / step_ms}}
    return res


def rq_step_flop(B, dims):
    """Algorithmic flops of one RQ-VAE training step (train.py:113-118): encoder + decoder GEMMs
    forward (2·B·in·out each) and backward (twice that: input and weight gradients)."""
    lin = sum(2 * B * i * o for i, o in zip(dims[:-1], dims[1:]))
    return 3 * 2 * lin


def _ref_rq_step(model, opt, x, use_sk=True):
    """RQ-VAE/train.py:110-118 as the reference writes it, in torch ops on any device: the torch
    MLPs, vq.py:63-99 per level (the [B, K] distance matrix, center_distance_for_constraint,
    layers.py:85-108's float64 Sinkhorn, argmax), compute_loss, backward, clip, step."""
    import torch.nn.functional as F
    opt.zero_grad()
    z = model.encoder.mlp_layers(x)
    res, x_q, losses = z, 0, []
    for q in model.rq.vq_layers:
        C = q.embedding.weight
        d = (res ** 2).sum(1, keepdim=True) + (C ** 2).sum(1, keepdim=True).t() - 2 * res @ C.t()
        if use_sk and q.sk_epsilon > 0:
            with torch.no_grad():
                mx, mn = d.max(), d.min()
                mid = (mx + mn) / 2
                amp = mx - mid + 1e-5
                assert amp > 0
                Q = torch.exp(-((d - mid) / amp).double() / q.sk_epsilon)
                Bq, Kq = Q.shape
                Q /= Q.sum(-1, keepdim=True).sum(-2, keepdim=True)
                for _ in range(q.sk_iters):
                    Q /= Q.sum(1, keepdim=True)
                    Q /= Bq
                    Q /= Q.sum(0, keepdim=True)
                    Q /= Kq
                Q *= Bq
                idx = Q.argmax(-1)
        else:
            idx = d.argmin(-1)
        xq = q.embedding(idx)
        losses.append(F.mse_loss(xq, res.detach()) + q.beta * F.mse_loss(xq.detach(), res))
        xq = res + (xq - res).detach()
        res = res - xq
        x_q = x_q + xq
    out = model.decoder.mlp_layers(x_q)
    loss = F.mse_loss(out, x) + model.quant_loss_weight * torch.stack(losses).mean()
    loss.backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
    opt.step()
    return loss


def bench_rq_train_step(a, world, rank, dev, cpu=False):
    """RQ-VAE/train.py:108-119 at main.py's configuration (batch 64, 768 -> [256, 128] -> 32,
    3 x 8 codebooks, Sinkhorn eps 0.01 x 50 iterations at every level, dropout 0.1, AdamW 1e-3 /
    1e-4, linear warm-up schedule): the captured step (ops.RqTrainGraph) against the same step op
    by op and the reference formulation on the same GPU."""
    import copy
    from transformers import get_linear_schedule_with_warmup
    from gr_amd import RQVAE
    B, dims = 64, [768, 256, 128, 32]
    torch.manual_seed(11 + rank)

    def make(capturable):
        m = RQVAE(in_dim=768, num_emb_list=[8, 8, 8], e_dim=32, layers=[256, 128], dropout_prob=0.1,
                  bn=False, loss_type="mse", quant_loss_weight=0.1, beta=0.25, kmeans_init=False,
                  kmeans_iters=50, sk_epsilons=[0.01] * 3, sk_iters=50)
        for q in m.rq.vq_layers:   # stands in for the k-means init of the first batch
            q.embedding.weight.data.normal_(0.0, 0.3)
        m = m.to(dev).train()
        if capturable:   # the drop-in's step: the fused AdamW kernel (capturable, tensor lr)
            o = torch.optim.AdamW(m.parameters(), lr=torch.tensor(1e-3, device=dev), weight_decay=1e-4,
                                  capturable=True, fused=True)
        else:            # train.py:56-63 as written (foreach AdamW)
            o = torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=1e-4)
        return m, o, get_linear_schedule_with_warmup(o, 10, 10_000)

    x = synth.items(B, 13 + rank, dev)   # BERT-statistics item embeddings
    m, o, sch = make(True)
    inputs = x.clone()
    step = ops.RqTrainGraph(m, o, inputs)

    def captured():
        step.replay()
        sch.step()
    wall, dev_ms = timed(captured, a.steps, a.warmup, world)
    m2, o2, sch2 = make(True)

    def eager():
        o2.zero_grad(set_to_none=True)
        out, rq_loss, _ = m2(x)
        loss, _ = m2.compute_loss(out, rq_loss, xs=x)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(m2.parameters(), 1.0)
        o2.step()
        sch2.step()
    e_wall, _ = timed(eager, a.steps, a.warmup, world)
    m3, o3, sch3 = make(False)

    def reference():
        _ref_rq_step(m3, o3, x)
        sch3.step()
    r_ms = kernel_ms(reference, reps=10)
    fl = rq_step_flop(B, dims) * 2   # encoder and decoder
    step_ms = wall / a.steps * 1e3
    res = {"metric": "train_steps_items/s", "value": B * world * a.steps / wall, "unit": "items/s",
           "ms_per_step": step_ms, "scaling": "weak",
           "config": {"workload": "rq_train_step: RQ-VAE train.py:108-119 whole step at main.py's configuration "
                                  "(batch 64, 768 -> [256,128] -> 32, 3x8 codebooks, Sinkhorn eps 0.01 x 50 "
                                  "iterations per level on the kernels, dropout 0.1, AdamW (fused, capturable), "
                                  "clip 1.0, linear warm-up schedule), one captured graph",
                      "items_per_rank_per_step": B, "parallelism": f"item-sharded x{world} (data parallel "
                                                                  f"without the gradient all-reduce)"},
           "roofline": {"bound": "mfma", "achieved": fl / (dev_ms * 1e-3) / 1e12, "peak": FP32_PEAK_TFLOPS,
                        "unit": "TFLOP/s", "frac": fl / (dev_ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS,
                        "traffic": None, "kernel": "whole step (latency-bound: batch 64)",
                        "flop_per_step": fl, "step_device_ms": dev_ms},
           "eager": {"note": "the same step issued op by op (kernel Sinkhorn, torch MLPs)",
                     "value": B * world * a.steps / e_wall, "ms_per_step": e_wall / a.steps * 1e3},
           "reference_formulation_gpu": {"note": "train.py:108-119 as written (torch distance matrix, float64 "
                                                 "Sinkhorn with its host-synchronising amplitude assert) on "
                                                 "the same GPU", "ms_per_step": r_ms, "speedup": r_ms / step_ms}}
    if cpu:
        mc = copy.deepcopy(m3).cpu()
        oc = torch.optim.AdamW(mc.parameters(), lr=1e-3, weight_decay=1e-4)
        xc = x.cpu()
        res["cpu_baseline"] = cpu_median(lambda: _ref_rq_step(mc, oc, xc), B, "items/s",
                                         "train.py:108-119 reference formulation, batch 64, main.py config")
    del step
    return res


def bench_c5_shard(a, table, h, targets, dev, shards=8):
    """The per-GPU work of the 8-GPU C5 point, timed on one GPU: 512 users against one catalog
    shard of 125,001 rows (rows [lo, hi) of the 1M-item ``table``; the first shard, which also masks
    row 0): the owner's target logits (gr_score_pairs_f32) + fused score + top-10 + strict counts
    (gr_score_topk_f32).  The collectives around it (all-reduce of B floats and B counts,
    all-gather of B x 10 candidates) are latency-bound and not included."""
    from gr_amd import dist as D
    d, B, k = h.shape[1], h.shape[0], 10
    lo, hi = D.shard_range(table.shape[0], 0, shards)
    shard = table[lo:hi]
    t = targets.reshape(-1)
    own = (t >= lo) & (t < hi)
    loc = torch.where(own, t - lo, torch.zeros_like(t))

    def step():
        ts = ops.score_pairs(h, shard, loc, mask_col0=(lo == 0))
        return ops.score_topk(h, shard, k, lo, thresholds=ts, mask_col0=(lo == 0))

    wall, dev_ms = timed(step, a.steps, a.warmup, 1)
    ts = ops.score_pairs(h, shard, loc, mask_col0=(lo == 0))
    topk_ms = kernel_ms(lambda: ops.score_topk(h, shard, k, lo, thresholds=ts, mask_col0=(lo == 0)))
    cnt_ms = kernel_ms(lambda: ops.score_count_gt(h, shard, ts, mask_col0=(lo == 0)))
    flop = 2 * d * (hi - lo) * B
    return {"metric": "seqs_scored/s", "value": B * a.steps / wall, "unit": "seqs/s",
            "ms_per_step": wall / a.steps * 1e3, "scaling": "per-rank shard of the 8-GPU C5 point",
            "config": {"workload": f"c5_shard: {B} users x one {hi - lo}-row catalog shard (1/{shards} of "
                                   f"{table.shape[0]}), d {d}, target logit + rank + top-{k}",
                       "rows": hi - lo, "users": B},
            "roofline": roofline(TOPK_PASS_HALF, flop, topk_ms, "shard",
                                 call_kernels=TOPK_CALL_KERNELS,
                                 note="one gr_score_topk_f32 call on the shard (all its launches: the tile "
                                      "pass with 16-row half-tile maxima, topk_half auto, + the select); flop "
                                      "counts the scoring GEMM once; traffic is the whole call's"),
            "call": {"device_ms": dev_ms, "score_topk_ms": topk_ms, "score_count_ms": cnt_ms,
                     "frac_of_fp32_peak_step": flop / (dev_ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS}}


def _one_rank_rccl(dev):
    """A one-rank RCCL process group on ``dev`` for a leg that needs collectives at N = 1 (None if
    one is already up -- then it is the caller's -- or RCCL fails to initialise; the error string
    is returned instead)."""
    if dist.is_initialized():
        return None
    try:
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=dev)
        return True
    except Exception as ex:   # reported in the leg, the rest of the bench continues
        return f"{type(ex).__name__}: {ex}"


def c5_rank_with_collectives(a, dev, W, B, d, k, lo, h, shard, t, own, loc, m0, forward, gathered):
    """rank 0's C5 step at N = ``W`` WITH its collectives, timed on one GPU
    through a one-rank RCCL group, every message at its N = W size (the all-gather of the [B, d]
    hidden states, the all-reduces of B target logits and B counts, the all-gather of the
    [W, B, 2k] packed candidates -- a one-rank all-gather moves its whole output):
      * serial_ms: the exchange as dist.sharded_rank_topk runs it (bench.py's pre-r6 N > 1 step);
      * overlapped_ms: as dist.sharded_rank_topk_batches runs it with P user sub-batches (the
        "split" form): the target all-reduce of sub-batch b+1 and the count all-reduce + candidate
        all-gather of sub-batch b run on RCCL's stream under sub-batch b+1's scoring;
      * xstep_ms: as dist.ShardedRankPipeline runs it (the "xstep" form): the whole batch scored in
        one launch, its count all-reduce + candidate all-gather under the NEXT step's forward.
    The messages' xGMI latency between ranks is not on one GPU: these are the collectives' issue,
    launch and local-copy costs at the real sizes, not the 8-GPU wall time."""
    from gr_amd import dist as D
    pg = _one_rank_rccl(dev)
    if isinstance(pg, str):
        return {"collectives_error": pg}
    if pg is None and (dist.get_backend() != "nccl" or dist.get_world_size() != 1):
        return {"collectives_error": f"an existing {dist.get_backend()} group of {dist.get_world_size()} ranks "
                                     "(the leg needs a one-rank RCCL group)"}
    try:
        hin = h.clone()
        hout = torch.empty_like(h)
        packed_in = gathered.clone().view(W * B, -1)

        def serial():
            forward()
            dist.all_gather_into_tensor(hout, hin)
            tl = torch.where(own, ops.score_pairs(hout, shard, loc, mask_col0=m0), torch.zeros_like(hout[:, 0]))
            dist.all_reduce(tl)
            v, i, c = ops.score_topk(hout, shard, k, lo, thresholds=tl, mask_col0=m0)
            dist.all_reduce(c)
            packed_in[:B].copy_(D._pack(v, i))
            gout = torch.empty((W, B, 2 * k), dtype=torch.int64, device=dev)
            dist.all_gather_into_tensor(gout.view(W * B, -1), packed_in)
            ops.merge_topk_packed(gout, W, k, k)
            return c + 1

        def overlapped_fn(P):
            cuts = [B * j // P for j in range(P + 1)]
            subs = list(zip(cuts[:-1], cuts[1:]))
            pins = [torch.stack([gathered[r, x:y] for r in range(W)]).contiguous() for x, y in subs]

            def step():
                forward()
                dist.all_gather_into_tensor(hout, hin)

                def tstart(j):
                    x, y = subs[j]
                    tl = torch.where(own[x:y], ops.score_pairs(hout[x:y], shard, loc[x:y], mask_col0=m0),
                                     torch.zeros_like(hout[x:y, 0]))
                    return tl, dist.all_reduce(tl, async_op=True)

                def sstart(j, st):
                    x, y = subs[j]
                    tl, w = st
                    w.wait()
                    v, i, c = ops.score_topk(hout[x:y], shard, k, lo, thresholds=tl, mask_col0=m0)
                    w1 = dist.all_reduce(c, async_op=True)
                    pins[j][0].copy_(D._pack(v, i))
                    gout = torch.empty_like(pins[j])
                    w2 = dist.all_gather_into_tensor(gout.view(-1, 2 * k), pins[j].view(-1, 2 * k), async_op=True)
                    return c, gout, w1, w2

                def finish(sc):
                    c, gout, w1, w2 = sc
                    w1.wait()
                    w2.wait()
                    ops.merge_topk_packed(gout, W, k, k)
                    return c + 1

                out, prev = [], None
                pend = tstart(0)
                for j in range(len(subs)):
                    cur = pend
                    if j + 1 < len(subs):
                        pend = tstart(j + 1)
                    sc = sstart(j, cur)
                    if prev is not None:
                        out.append(finish(prev))
                    prev = sc
                out.append(finish(prev))
                return out
            return step

        xs = {"prev": None, "j": 0}
        xpins = [packed_in, packed_in.clone()]

        def xflush():
            prev, xs["prev"] = xs["prev"], None
            if prev is None:
                return None
            c, gout, w1, w2 = prev
            w1.wait()
            w2.wait()
            ops.merge_topk_packed(gout, W, k, k)
            return c + 1

        def xstep():   # as dist.ShardedRankPipeline runs it: the exchange under the next step's forward
            forward()
            dist.all_gather_into_tensor(hout, hin)
            tl = torch.where(own, ops.score_pairs(hout, shard, loc, mask_col0=m0), torch.zeros_like(hout[:, 0]))
            dist.all_reduce(tl)
            v, i, c = ops.score_topk(hout, shard, k, lo, thresholds=tl, mask_col0=m0)
            w1 = dist.all_reduce(c, async_op=True)
            pin = xpins[xs["j"] & 1]
            xs["j"] += 1
            pin[:B].copy_(D._pack(v, i))
            gout = torch.empty((W, B, 2 * k), dtype=torch.int64, device=dev)
            w2 = dist.all_gather_into_tensor(gout.view(W * B, -1), pin, async_op=True)
            out = xflush()
            xs["prev"] = (c, gout, w1, w2)
            return out

        steps_ = max(2, min(a.steps, 10))
        _, ser_ms = timed(serial, steps_, 2, 1)
        res = {"serial_ms": ser_ms, "serial_value": B / (ser_ms * 1e-3)}
        best = None
        for P in (2, 4):
            _, o_ms = timed(overlapped_fn(P), steps_, 2, 1)
            res[f"overlapped_ms_p{P}"] = o_ms
            if best is None or o_ms < best[1]:
                best = (P, o_ms)
        P_def = C5_PIPELINE_DEFAULT
        _, x_ms = timed(xstep, steps_, 2, 1, tail=xflush)
        forms = {"serial": ser_ms, "split": res.get(f"overlapped_ms_p{P_def}", best[1]), "xstep": x_ms}
        res.update({"overlapped_ms": forms["split"], "overlapped_pipeline": P_def,
                    "overlapped_value": B / (forms["split"] * 1e-3),
                    "xstep_ms": x_ms, "xstep_value": B / (x_ms * 1e-3),
                    "exchange_best": min(forms, key=forms.get),
                    "collectives_backend": "nccl (RCCL), one-rank group, N = %d message sizes" % W})
        return res
    finally:
        if pg is True:
            dist.destroy_process_group()


def bench_c5_rank(a, dev):
    """the per-rank unit of the N-GPU C5 point (N = ``--c5-rank-world``, 8),
    timed on one GPU.  Rank 0's step of ``bench_sas_c5`` at world N: the transformer forward of its
    own c5_batch users, then -- on the all-gathered hidden states of all B = c5_batch x N users --
    the owner's target logits (gr_score_pairs_f32), the fused strict count + local top-10 over its
    catalog shard (rows [0, (items+1)/N), which also masks row 0; gr_score_topk_f32) and the merge of
    the N x 10 gathered candidates (gr_merge_topk_packed).  The collectives themselves (all-gather of
    B x d floats, two all-reduces of B scalars, all-gather of B x 10 candidates: about 2.4 MB per
    rank at N = 8) are not on one GPU; ``collective_bytes_per_rank`` states them.  ``value`` = the B
    users of one N-GPU step / this rank's device time per step: the N-GPU throughput when the
    collectives overlap the scoring."""
    from gr_amd import dist as D
    W = a.c5_rank_world
    d, n, items, k = 128, 200, a.c5_items, 10
    B = a.c5_batch * W
    p = synth.sasrec_params(d, n, 2, 1, 64, dev)
    seqs = synth.sequences(B, n, items, 5000, dev)
    targets = torch.randint(1, items + 1, (B,), generator=torch.Generator(device=dev).manual_seed(6), device=dev)
    lo, hi = D.shard_range(items + 1, 0, W)
    shard = synth.table_rows(torch.arange(lo, hi, device=dev), d, 7, dev)
    hs = []
    for r in range(W):   # every rank's hidden states (what the all-gather delivers), built once
        ulo, uhi = D.shard_range(B, r, W)
        mr, sr = synth.sasrec_rank_model(items, p, seqs[ulo:uhi], dev, seed=5)
        hs.append(mr.last_hidden(sr))
        if r == 0:
            model, lseqs = mr, sr
    h = torch.cat(hs)
    del hs
    t = targets
    own = (t >= lo) & (t < hi)
    loc = torch.where(own, t - lo, torch.zeros_like(t))
    m0 = lo == 0
    # the other ranks' candidates: this shard's lists with ids moved into their shards (the merge's
    # cost depends on the [B, N k] shape, not on the values)
    _, v0, i0 = D.sharded_rank_topk(h, shard, lo, targets, k=k)
    gathered = torch.stack([D._pack(v0, i0 + D.shard_range(items + 1, r, W)[0]) for r in range(W)])

    def forward():
        return model.last_hidden(lseqs)

    def pairs():
        return torch.where(own, ops.score_pairs(h, shard, loc, mask_col0=m0), torch.zeros_like(h[:, 0]))

    ts = pairs()

    def topk():
        return ops.score_topk(h, shard, k, lo, thresholds=ts, mask_col0=m0)

    def merge():   # what dist._exchange runs on the all-gathered [W, B, 2k] buffer
        return ops.merge_topk_packed(gathered, W, k, k)

    def step():
        forward()
        tl = pairs()
        _, _, c = ops.score_topk(h, shard, k, lo, thresholds=tl, mask_col0=m0)
        merge()
        return c + 1

    steps_ = max(2, min(a.steps, 10))
    wall, dev_ms = timed(step, steps_, 2, 1)
    split = {"forward_ms": kernel_ms(forward), "score_pairs_ms": kernel_ms(pairs),
             "score_topk_ms": kernel_ms(topk), "merge_topk_ms": kernel_ms(merge)}
    fl_topk = 2 * d * (hi - lo) * B
    coll = B * d * 4 + B * 4 + B * 8 + B * k * 16
    colls = c5_rank_with_collectives(a, dev, W, B, d, k, lo, h, shard, t, own, loc, m0, forward, gathered)
    # the step bench.py's N > 1 run picks automatically: the faster of the serial and pipelined
    # exchange (bench_sas_c5's probe)
    val_ms = min(colls.get("serial_ms") or dev_ms, colls.get("overlapped_ms") or dev_ms,
                 colls.get("xstep_ms") or dev_ms)
    return {"metric": "seqs_scored/s", "value": B / (val_ms * 1e-3), "unit": "seqs/s",
            "scaling": f"one rank of the N = {W} C5 point, projected to the whole job",
            "ms_per_step": val_ms, "wall_ms_per_step": wall / steps_ * 1e3,
            "config": {"workload": f"c5_rank: rank 0 of N = {W}: forward of {B // W} users (d {d}, n {n}), "
                                   f"target logits + rank + top-{k} of all {B} users on rows [{lo}, {hi}) "
                                   f"of the {items + 1}-row catalog, merge of {W} x {k} candidates",
                       "users_per_step": B, "users_forwarded": B // W, "rows": hi - lo},
            "projected_value_note": f"value = the {B} users of one N = {W} step / this rank's step time WITH "
                                    f"its collectives: min(serial_ms, overlapped_ms, xstep_ms), the exchange bench.py's "
                                    f"N > 1 run selects by timing both (every collective at its N = {W} message "
                                    f"size through a one-rank RCCL group; xGMI latency between ranks is not on "
                                    f"one GPU). no_collectives_ms: the kernels alone",
            "no_collectives_ms": dev_ms, "no_collectives_value": B / (dev_ms * 1e-3),
            **colls,
            "collective_bytes_per_rank": coll,
            "split": split,
            "roofline": roofline("score_topk_kernel<128,10,", fl_topk, split["score_topk_ms"], "c5_rank",
                                 call_kernels=TOPK_CALL_KERNELS,
                                 note=f"one gr_score_topk_f32 call of {B} users on the {hi - lo}-row shard"),
            "call": {"device_ms": dev_ms,
                     "flop_per_step": sas_exec_flop_per_user(d, n, -1, causal=True, tail_h=True) * (B // W) + fl_topk,
                     "frac_of_fp32_peak_executed": (sas_exec_flop_per_user(d, n, -1, causal=True, tail_h=True) * (B // W)
                                                    + fl_topk) / (dev_ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS}}


def bench_ref_eval(a, dev, cpu):
    """VERDICT r4 missing #1: SASRec/evaluate.py at the reference's own deployed configuration
    (SASRec/main.py: d 16, max_len 20, 2 blocks, 1 head, mlp 64; the 706-course catalog; the 95,423
    test users of SASRec/logs/sasrec.log; eval_batch_size 128), synthetic sequences / targets and
    seeded weights.  The whole evaluation: the fused rank of every batch of 128 users (evaluate.py:
    26-32 without logits: last_hidden + gr_score_pairs_f32 + gr_score_count_gt_f32 at d 16), then
    HR@10 / NDCG@10 on the host as evaluate.py:35-47 does; also the same users in one call."""
    from gr_amd import evaluate as E
    items, n, d, users, bs = 706, 20, 16, 95_423, 128
    p = synth.sasrec_params(d, n, 2, 1, 64, dev)
    model = synth.sasrec_model(items, p, dev, seed=16)
    seqs = synth.sequences(users, n, items, 9000, dev)
    tg = torch.randint(1, items + 1, (users,), generator=torch.Generator(device=dev).manual_seed(10), device=dev)

    def run(b):
        return torch.cat([E.rank_batch(model, seqs[i:i + b], tg[i:i + b]) for i in range(0, users, b)])

    def whole(b):
        r = run(b)
        return E.hr_ndcg(r.cpu().numpy(), 10)   # host float64 metric (evaluate.py:35-47)

    spinup(lambda: run(bs), 0.5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        hr, nd = whole(bs)
    wall = (time.perf_counter() - t0) / reps
    one_ms = kernel_ms(lambda: run(users), reps=20)
    batch_ms = kernel_ms(lambda: run(bs), reps=5)
    res = {"metric": "eval_users/s", "value": users / wall, "unit": "users/s", "ms_per_eval": wall * 1e3,
           "config": {"workload": f"ref_eval: SASRec/evaluate.py at SASRec/main.py's configuration (d {d}, "
                                  f"max_len {n}, 2 blocks, 1 head, mlp 64), {items}-item catalog, {users} test "
                                  f"users in batches of {bs}, fused rank (no logits) + host HR/NDCG@10",
                      "users": users, "batch": bs},
           "hr10": hr, "ndcg10": nd,
           "device_ms_batches_of_128": batch_ms, "device_ms_one_call": one_ms,
           "one_call_users_per_s": users / (one_ms * 1e-3),
           "note": "latency-bound at this size (746 batches of 128 users, 707-row table): the value is the "
                   "whole evaluation incl. the host metric; device_ms_one_call scores every user in one call"}
    if cpu:
        from oracle import sasrec_oracle
        sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
        sample = 8192
        sc, tc = seqs[:sample].cpu(), tg[:sample].cpu()

        def cpu_eval():   # evaluate.py:26-32 on the restatement, batches of 128
            out = []
            for i in range(0, sample, bs):
                lg = sasrec_oracle.predict(sc[i:i + bs], sd, 2, 1, 1e-8)
                lg[:, 0] = -1e9
                t = lg.gather(1, tc[i:i + bs, None])
                out.append((lg > t).sum(1) + 1)
            return torch.cat(out)
        gpu_r = run(bs)[:sample].cpu()
        res["cpu_baseline"] = cpu_median(cpu_eval, sample, "users/s",
                                         f"oracle/sasrec_oracle.predict + the evaluate.py:27-32 rank, {sample} of "
                                         f"the users in batches of {bs}", warm=1, reps=3,
                                         agree=lambda r: {"users": sample, "ranks_differ": int((r != gpu_r).sum()),
                                                          "hr10_cpu": float((r <= 10).double().mean()),
                                                          "hr10_gpu": float((gpu_r <= 10).double().mean())})
    return res


def _call_pattern(fn, units, reps=200):
    """Per-call cost of a small drop-in call at the reference's own batch size: host time to issue
    one call (no sync), time of one isolated call (HIP events around it: includes the wait for the
    host's launches), the pipelined wall time per call (``reps`` calls back to back, one sync at the
    end), and the device time per call of 20 calls replayed as one captured graph."""
    spinup(fn, 0.3)
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for _ in range(reps):
        t1 = time.perf_counter()
        fn()
        host.append(time.perf_counter() - t1)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
    for s_, e_ in ev:
        torch.cuda.synchronize()
        s_.record()
        fn()
        e_.record()
    torch.cuda.synchronize()
    dev_us = float(np.median([s_.elapsed_time(e_) for s_, e_ in ev])) * 1e3
    # the GPU's own time per call: 20 calls captured as one graph and replayed (no host issue time;
    # device_us_per_call above times one isolated call, which waits for the host's launches)
    graph_us = None
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(20):
                fn()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        graph_us = e0.elapsed_time(e1) / 200 * 1e3
        del g
    except Exception as ex:   # a call that cannot be captured: reported as such
        graph_us = f"not capturable: {type(ex).__name__}"
    return {"value": units / wall, "us_per_call": wall * 1e6, "host_us_per_call": float(np.median(host)) * 1e6,
            "device_us_per_call": dev_us, "graph_us_per_call": graph_us}


def bench_calls(rq_model, sas_model, sas_n, sas_items, dev, cpu=True):
    """the drop-in methods at the reference's own call sizes, host overhead
    included: ``model.get_indices(x[:64])`` (RQ-VAE/infer.py:84-95, batch 64) and
    ``model.predict(seqs[:128])`` + the evaluate tail (SASRec/evaluate.py:13, 26-32, batch 128)."""
    from gr_amd import evaluate as E
    out = {}
    x = synth.items(64, 77, dev)
    r = _call_pattern(lambda: rq_model.get_indices(x), 64)
    r.update(unit="items/s", workload="RQVAE.get_indices(x[64, 768]) at C2 weights")
    if cpu:
        r["cpu_baseline"] = cpu_rq_baseline(rq_model, 64, "batch 64 (infer.py:84)")
    out["rq_get_indices_b64"] = r
    if sas_model is not None:
        seqs = synth.sequences(128, sas_n, sas_items, 78, dev)
        tg = torch.randint(1, sas_items + 1, (128,), generator=torch.Generator(device=dev).manual_seed(9), device=dev)
        r = _call_pattern(lambda: sas_model.predict(seqs), 128)
        r.update(unit="seqs/s", workload=f"SASRec.predict(seqs[128, {sas_n}]) at C3 weights, logits written")
        if cpu:
            r["cpu_baseline"] = cpu_sas_baseline(sas_model, 128, sas_n, sas_items, "batch 128 (evaluate.py:13)")
        out["sas_predict_b128"] = r
        r = _call_pattern(lambda: E.rank_batch(sas_model, seqs, tg), 128)
        r.update(unit="seqs/s", workload="evaluate.rank_batch at batch 128: forward + target logit + strict "
                                         "count (evaluate.py:26-32 without the logits)")
        out["sas_rank_b128"] = r
    return out


LEGS = ["c2", "calls", "ref_eval", "sasrec", "c4", "c5", "shard", "c5_rank", "train", "train_step", "rq_train_step"]
OPT_LEGS = []   # run only when named in --legs


def selftest(a, world, rank):
    """GR_BENCH_DEVICE=cpu: the multi-rank plumbing of this bench on CPU ranks over gloo -- the
    process group, max-over-ranks timing, per-rank reporting and the C5 result checksum agreement
    -- with a deterministic stand-in for the merged C5 result (no GPU, no kernels)."""
    global COLL_DEV
    COLL_DEV = "cpu"
    if world > 1:
        dist.init_process_group("gloo")
    g = torch.Generator().manual_seed(0)   # the same "merged" result on every rank, as after C5's exchange
    ranks = torch.randint(1, 1000, (512,), generator=g)
    vals = torch.randn(512, 10, generator=g)
    ids = torch.randint(1, 10**6, (512, 10), generator=g)
    t0 = time.perf_counter()
    x = torch.randn(256, 256, generator=g)
    for _ in range(a.steps):
        x = torch.tanh(x @ x.t() / 256)
    wall = time.perf_counter() - t0
    walls = per_rank(wall, world)
    line = {"metric": METRIC, "value": None, "unit": "items/s", "n_gpus": world, "steps": a.steps,
            "note": "launcher self-test (GR_BENCH_DEVICE=cpu): no GPU work was measured",
            "selftest": {"wall_s_per_rank": walls, "max_wall_s": max(walls),
                         "result_checksum": result_checksum((ranks, vals, ids), world)}}
    line["dist"] = ({"backend": str(dist.get_backend()), "world_size": dist.get_world_size()}
                    if dist.is_initialized() else {"backend": None, "world_size": 1})
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def main():
    a = parse()
    global SPINUP_S
    SPINUP_S = a.spinup_s
    legs = [l for l in (a.legs.split(",") if a.legs else LEGS) if l]
    skip = set(s for s in a.skip.split(",") if s)
    legs = [l for l in legs if l not in skip]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world and world == 1 and a.gpus > 1:
        sys.exit("bench.py: --gpus N>1 without WORLD_SIZE: run it as a script (it launches its ranks)")
    if os.environ.get("GR_BENCH_DEVICE") == "cpu":   # launcher / process-group self-test, no GPU
        return selftest(a, world, rank)
    # GR_BENCH_BACKEND=gloo is a rehearsal mode only (several ranks sharing one GPU to exercise the
    # multi-rank code paths on a one-GPU box); real runs use RCCL ("nccl"), one GPU per rank.
    backend = os.environ.get("GR_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # GR_BENCH_PG=1: a process group even for one rank (torchrun --nproc-per-node 1), so a one-GPU
    # box runs the C5 exchange's collectives through RCCL exactly as the 8-GPU node does
    if world > 1 or os.environ.get("GR_BENCH_PG") == "1":
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    cpu = rank == 0 and world == 1 and not a.no_cpu_baseline

    if "c2" in legs:
        line, rq_model = bench_rq_c2(a, world, rank, dev)
        if cpu:
            line["cpu_baseline"] = cpu_rq_baseline(rq_model, 100_000, "C2")
    else:   # a partial run (per-leg profiling): the headline leg is not measured
        line = {"metric": METRIC, "value": None, "unit": "items/s", "n_gpus": world, "legs": legs,
                "note": "partial run (--legs): the C2 headline was not measured"}
        rq_model = synth.rqvae_model(3, 256, dev) if "calls" in legs else None
    sas_model, sn, sitems = None, 50, 100_000
    if "sasrec" in legs or "calls" in legs:
        sres, sas_model, (sn, sitems) = bench_sas_c3(a, world, rank, dev)
        if "sasrec" in legs:
            line["sasrec"] = sres
            if cpu:
                line["sasrec"]["cpu_baseline"] = cpu_sas_baseline(sas_model, 1024, sn, sitems, "C3")
    if "calls" in legs and world == 1:
        line["calls"] = bench_calls(rq_model, sas_model, sn, sitems, dev, cpu)
    if "ref_eval" in legs and world == 1:
        line["ref_eval"] = bench_ref_eval(a, dev, cpu)
    if "c4" in legs:
        line["rq_c4"], c4_model = bench_rq_c4(a, world, rank, dev)
        if cpu:
            line["rq_c4"]["cpu_baseline"] = cpu_rq_baseline(c4_model, 20_000, "C4 sample")
        del c4_model
        torch.cuda.empty_cache()
    if "c5" in legs or "shard" in legs:
        c5, c5_model, h5, t5, table5 = bench_sas_c5(a, world, rank, dev, time_it="c5" in legs)
        if "c5" in legs:
            line["sasrec_c5"] = c5
            if cpu:   # at N = 1 the rank's shard is the whole table
                line["sasrec_c5"]["cpu_baseline"] = cpu_sas_baseline(
                    c5_model, 128, 200, a.c5_items, "C5", table=table5,
                    params=synth.sasrec_params(128, 200, 2, 1, 64, dev))
        if "shard" in legs and world == 1:
            line["c5_shard"] = bench_c5_shard(a, table5, h5, t5, dev)
        del c5_model, h5, table5
        torch.cuda.empty_cache()
    if "c5_rank" in legs and world == 1:
        line["c5_rank"] = bench_c5_rank(a, dev)
        torch.cuda.empty_cache()
    if "train_step" in legs:
        line["sasrec_train_step"] = bench_sas_train_step(a, world, rank, dev)
    if "rq_train_step" in legs:
        line["rq_train_step"] = bench_rq_train_step(a, world, rank, dev, cpu)
    if "train" in legs:
        line["sasrec_train"] = bench_sas_train(a, world, rank, dev)
    # what the process group saw, so a multi-GPU line proves its ranks took part
    if dist.is_initialized():
        devs = per_rank(float(local), world)
        line["dist"] = {"backend": str(dist.get_backend()), "world_size": dist.get_world_size(),
                        "local_device_per_rank": [int(x) for x in devs],
                        "device_name": torch.cuda.get_device_name(dev)}
    else:
        line["dist"] = {"backend": None, "world_size": 1, "note": "no process group (N = 1)"}
    # every leg's headline number once more at the END of the line, where a truncated log tail shows it
    summ = {}
    for key, name in (("value", "c2_items_per_s"),):
        if line.get(key) is not None:
            summ[name] = line[key]
    for leg, name in (("sasrec", "c3_seqs_per_s"), ("rq_c4", "c4_items_per_s"), ("sasrec_c5", "c5_seqs_per_s"),
                      ("c5_shard", "c5_shard_seqs_per_s"), ("c5_rank", "c5_rank_projected_seqs_per_s"),
                      ("ref_eval", "ref_eval_users_per_s"), ("sasrec_train_step", "sasrec_train_step_seqs_per_s"),
                      ("rq_train_step", "rq_train_step_items_per_s"), ("sasrec_train", "sasrec_train_seqs_per_s")):
        if isinstance(line.get(leg), dict) and line[leg].get("value") is not None:
            summ[name] = line[leg]["value"]
    # the bench host's CPU-path disagreement, characterised, where the tail shows it
    for tag, obj in (("c2", line), ("c4", line.get("rq_c4") or {})):
        ag = (obj.get("cpu_baseline") or {}).get("agreement") or {}
        if "rows_ids_differ" in ag:
            summ[f"{tag}_host_rows"] = ag["rows"]
            summ[f"{tag}_host_rows_differ"] = ag["rows_ids_differ"]
            if "rows_ids_differ_unflagged" in ag:
                summ[f"{tag}_host_rows_differ_unflagged"] = ag["rows_ids_differ_unflagged"]
                summ[f"{tag}_host_dz_over_z_max"] = ag["host_dz_over_z_max"]
    for key in ("serial_ms", "overlapped_ms", "xstep_ms"):
        if isinstance(line.get("c5_rank"), dict) and key in line["c5_rank"]:
            summ[f"c5_rank_{key}"] = line["c5_rank"][key]
    rf = line.get("sasrec", {}).get("roofline") if isinstance(line.get("sasrec"), dict) else None
    if isinstance(rf, dict):   # both figures of the C3 scoring kernel
        summ["c3_score_frac_event"] = rf.get("frac")
        if "frac_rocprof" in rf:
            summ["c3_score_frac_rocprof"] = rf["frac_rocprof"]
    line["summary"] = summ
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
