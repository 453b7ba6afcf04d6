"""bench.py's multi-rank launch (CPU, gloo): `--gpus N` with no torch.distributed environment
starts N ranks as one child torch.distributed.run, every rank joins one process group of N,
and rank 0's JSON line reports n_gpus = N with the backend. `--dry-run` stops before any GPU
work (one all-reduce of a gradient-sized buffer), so this runs in the CPU suite; on the GPU
box the same launch path carries the real step over RCCL."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*args, env=None):
    e = dict(os.environ, OMP_NUM_THREADS="1")
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=e,
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    return p


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_spawns_n_ranks(n):
    p = run_bench("--gpus", str(n), "--dry-run", "--backend", "gloo")
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == n
    assert out["dist"] == {"backend": "gloo", "world_size": n}
    assert out["config"]["parallelism"] == f"dp{n}"
    assert out["allreduce_ok"] is True


def test_single_rank_default():
    p = run_bench("--dry-run")
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["n_gpus"] == 1 and out["dist"]["world_size"] == 1


def test_world_size_mismatch_refused():
    """Under an external launcher the rank count must equal --gpus (no silent dp1 result)."""
    p = run_bench("--gpus", "4", "--dry-run",
                  env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE=2" in (p.stderr + p.stdout)


def test_pmc_traffic_prefers_the_workloads_own_pass():
    """bench.pmc_traffic: a "<workload>:<kernel>" key (the PMC pass recorded for that workload)
    wins over the bare kernel name, which stays the fallback; unknown kernels give (None, None).
    Every kernel the committed traffic table names resolves with its source file present."""
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench

    table = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))
    for key, v in table.items():
        assert v["bytes_per_launch"] > 0
        fname = v["source"].split(" ")[0]  # a note may follow the file name
        assert os.path.exists(os.path.join(ROOT, "profiles", fname)), v["source"]
    bare = [k for k in table if ":" not in k.split("(")[0]]
    wl = [k for k in table if ":" in k.split("(")[0]]
    assert bare and wl
    k = wl[0]
    w, kern = k.split(":", 1)
    b, src = bench.pmc_traffic(kern, w)
    assert (b, src) == (table[k]["bytes_per_launch"], table[k]["source"])
    b0, src0 = bench.pmc_traffic(bare[0])
    assert (b0, src0) == (table[bare[0]]["bytes_per_launch"], table[bare[0]]["source"])
    assert bench.pmc_traffic("no_such_kernel", "c2") == (None, None)
