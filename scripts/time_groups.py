"""Wall time per call of the grouped (collision-group) encoder at two group-size mixes: many 2-5-row groups
(the per-row kernel) and 16-128-row groups (one MFMA-kernel call when their orders agree)."""
import sys, time, torch, numpy as np
sys.path.insert(0, "tests/golden"); sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import golden_lib as gl
from test_rq_gpu import build_model
dev = torch.device("cuda:0")
x, sd, _, meta = gl.rq_inputs("rq_syn_3x256")
m = build_model(meta, sd, dev)
rng = np.random.default_rng(5)
from gr_amd import ops
real_plan = ops.mkl_plan
for label, sizes in (("groups 2-5 x 400", [int(v) for v in rng.integers(2, 6, 400)]),
                     ("groups 16-128 x 40", [int(v) for v in rng.integers(16, 129, 40)])):
    xs = torch.from_numpy(x[: sum(sizes)]).to(dev)
    res = {}
    for mode in ("every group on the per-row kernel", "chain-order groups batched"):
        # the first mode hides the chain plans, so every group takes the per-row kernel (the old path)
        ops.mkl_plan = (lambda m_, k_, n_: ("small16", 0, True)) if mode.startswith("every") else real_plan
        for _ in range(3):
            z = m.encoder(xs, group_sizes=sizes)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            z = m.encoder(xs, group_sizes=sizes)
        torch.cuda.synchronize()
        res[mode] = z.clone()
        print(f"{label}: {sum(sizes)} rows, {mode}: {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms per call", flush=True)
    a, b = res.values()
    print(f"{label}: outputs bitwise equal: {torch.equal(a, b)}", flush=True)
