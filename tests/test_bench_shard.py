"""The multi-GPU path of bench.py on CPU: world_size-2 gloo.

bench.py shards objects round-robin over ranks with no data-path collective
(SURVEY.md 8(e)); the only collective is the MAX over ranks of the timings.
These tests run that logic in two gloo processes (127.0.0.1 rendezvous).
"""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, per_rank, q):
    import torch.distributed as dist
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    owned = bench.owned_objects(rank, world, per_rank)
    # rank-dependent timings: the job time is the slowest rank's
    got = bench.max_over_ranks([1.0 + rank, 10.0 - rank, 5.0], dist, "cpu")
    objects = int(-bench.max_over_ranks([-(per_rank + rank)], dist, "cpu")[0])
    q.put((rank, owned, got, objects))
    dist.barrier()
    dist.destroy_process_group()


def test_owned_objects_partition():
    import bench
    for world in (1, 2, 4, 8):
        allo = sorted(o for r in range(world) for o in bench.owned_objects(r, world, 5))
        assert allo == list(range(5 * world))


@pytest.mark.timeout(120)
def test_gloo_world2_sharding_and_max():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, 3, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=90) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    (r0, own0, got0, n0), (r1, own1, got1, n1) = res
    assert own0 == [0, 2, 4] and own1 == [1, 3, 5]          # object o -> rank o % 2, disjoint
    assert got0 == got1 == [2.0, 10.0, 5.0]                  # element-wise MAX over ranks
    assert n0 == n1 == 3                                     # both ranks run the minimum count


def test_parent_builds_before_ranks_start(monkeypatch):
    """bench.py --gpus N builds the library once in the parent (no GPU
    touched) before torchrun starts the ranks, so the ranks find it fresh."""
    import bench
    from vds_amd import build as vbuild
    seen = {}

    def fake_relaunch(args):
        seen["stale_at_launch"] = vbuild._stale(vbuild.LIB)
        seen["gpus"] = args.gpus
        return 0

    monkeypatch.setattr(bench, "relaunch_with_torchrun", fake_relaunch)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 0
    assert seen == {"stale_at_launch": False, "gpus": 2}
