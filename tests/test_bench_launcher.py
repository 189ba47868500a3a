"""bench.py --gpus N self-launch: the same command form the driver uses for the
1-GPU BENCH line, ``python bench.py --gpus N``, starts its N ranks through torch.distributed.run and
prints one JSON line from rank 0.  Here on CPU ranks over gloo (GR_BENCH_DEVICE=cpu: the launcher,
the process group, max-over-ranks timing and the C5 checksum agreement; no kernels)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n):
    env = dict(os.environ, GR_BENCH_DEVICE="cpu", OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "LOCAL_RANK", "RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "2"],
                       env=env, cwd="/tmp", capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    return lines[0]


def test_bench_self_launches_two_ranks():
    line = _run(2)
    assert line["n_gpus"] == 2 and line["dist"] == {"backend": "gloo", "world_size": 2}
    st = line["selftest"]
    assert len(st["wall_s_per_rank"]) == 2 and st["max_wall_s"] == max(st["wall_s_per_rank"])
    assert st["result_checksum"]["ranks_agree"] and st["result_checksum"]["n_ranks_reporting"] == 2


def test_bench_one_rank_needs_no_launcher():
    line = _run(1)
    assert line["n_gpus"] == 1 and line["dist"]["world_size"] == 1
    # the checksum is independent of the world size (the same bits at N = 1 and N = 2)
    assert line["selftest"]["result_checksum"]["sha256_16"] == _run(2)["selftest"]["result_checksum"]["sha256_16"]
