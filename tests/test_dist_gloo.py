"""Multi-rank path on CPU: stripe sharding covers every stripe exactly once and
the benchmark's barrier / max-over-ranks reduction works under gloo with
world_size 2 (the N>1 bench path, without a GPU)."""
import os
import socket
import subprocess
import sys

import pytest

from nexoedge_amd.dist import shard_range

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shard_range_partitions():
    for total in (0, 1, 7, 4096, 4097, 10**6 + 3):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                lo, hi = shard_range(total, r, world)
                assert 0 <= lo <= hi <= total
                seen.extend(range(lo, hi)) if total < 10000 else seen.append((lo, hi))
            if total < 10000:
                assert seen == list(range(total))
            else:
                assert seen[0][0] == 0 and seen[-1][1] == total
                assert all(a[1] == b[0] for a, b in zip(seen, seen[1:]))
            sizes = [hi - lo for lo, hi in (shard_range(total, r, world) for r in range(world))]
            assert max(sizes) - min(sizes) <= 1


WORKER = r"""
import os, sys, time
sys.path.insert(0, {root!r})
from nexoedge_amd.dist import RankGroup, shard_range
g = RankGroup()
lo, hi = shard_range(4096, g.rank, g.world)
g.barrier()
t = 0.010 * (g.rank + 1)          # pretend rank r took (r+1)*10 ms
mx = g.max(t)
tot = g.sum(hi - lo)
nodes = ",".join(str(int(x)) for x in g.gather(3 - g.rank))  # e.g. each rank's NUMA node (bench.py)
print(f"rank={{g.rank}} world={{g.world}} lo={{lo}} hi={{hi}} max={{mx:.3f}} total={{tot:.0f}} nodes={{nodes}}", flush=True)
g.close()
"""


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_group_shard_matches_rank_sharding():
    """The in-process multi-GPU group (nxec_group_*) splits stripes exactly like
    the one-process-per-GPU ranks do, so both deployments code the same ranges."""
    from nexoedge_amd import nxec

    for total in (0, 1, 7, 4096, 4097, 10**6 + 3):
        for world in (1, 2, 3, 8):
            for r in range(world):
                lo, hi = shard_range(total, r, world)
                assert nxec.Group.shard(total, world, r) == (lo, hi - lo)


def test_group_without_device_fails_loudly():
    import pytest

    from nexoedge_amd import nxec

    try:
        import torch

        if torch.cuda.device_count() > 0:
            pytest.skip("a device is present")
    except ImportError:
        pass
    with pytest.raises(nxec.NxecError):
        nxec.Group([0, 0])


def test_gloo_world2_reduction(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(WORKER.format(root=ROOT))
    port = free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=180) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
    lines = sorted(l for o, _ in outs for l in o.splitlines() if l.startswith("rank="))
    assert lines[0] == "rank=0 world=2 lo=0 hi=2048 max=0.020 total=4096 nodes=3,2"
    assert lines[1] == "rank=1 world=2 lo=2048 hi=4096 max=0.020 total=4096 nodes=3,2"


def _bench(args, env_extra=None, timeout=240):
    env = dict(os.environ, **(env_extra or {}))
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(v, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


@pytest.mark.parametrize("world", [2, 8])
def test_bench_launches_ranks_itself(world):
    """`bench.py --gpus N` without torch.distributed.run starts N rank
    processes (gloo rendezvous on 127.0.0.1) and prints rank 0's single line
    with n_gpus = N (dry run: no GPU work); N = 8 is the driver's node."""
    import json

    r = _bench(["--gpus", str(world), "--dry-run", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["ranks_seen"] == world and d["steps"] == 3
    assert abs(d["max_elapsed_s"] - 0.001 * world) < 1e-9  # max over ranks, not rank 0's own value


def test_bench_launcher_fails_when_a_rank_fails():
    r = _bench(["--gpus", "2", "--dry-run"], {"NXEC_DRY_RUN_FAIL_RANK": "1"})
    assert r.returncode != 0
    assert "rank 1 exited with status 3" in r.stderr


def test_bench_under_torch_distributed_run_world8():
    """The driver's own N = 8 launch: `python -m torch.distributed.run
    --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 ... bench.py --gpus 8`
    (dry run: rendezvous, barrier, max-over-ranks and sums, one JSON line)."""
    import json

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(v, None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "8", "--dry-run", "--steps", "4", "--warmup", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip().startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["ranks_seen"] == 8 and abs(d["max_elapsed_s"] - 0.008) < 1e-9


def test_bench_group_flag_dry_run():
    """`bench.py --gpus 8 --group` (the one-process nxec_group deployment
    measured beside the ranks): the dry run rendezvouses the 8 ranks and rank 0
    reports the group's plan -- 8 members, member i on device i, each with its
    own stripe batch -- in the same single line."""
    import json

    r = _bench(["--gpus", "8", "--group", "--dry-run", "--stripes", "512", "--steps", "2", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["ranks_seen"] == 8
    assert d["group"] == {"members": 8, "devices": list(range(8)), "stripes_per_member": 512}
