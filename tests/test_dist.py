"""CPU, world_size 2 over gloo: the multi-GPU path of bench.py -- round-robin
packet shards with no data-path collective, a barrier and a MAX-reduce of the
timing -- computed here with the CPU oracle as the per-rank worker."""
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root / "roce-sim_amd"))
    sys.path.insert(0, str(root / "oracle"))
    import torch
    import icrc_oracle as o
    from roce_icrc import synth
    dist.init_process_group("gloo", rank=rank, world_size=world)
    buf, stride, flen = synth.uniform_frames(n, 64, seed=100 + rank, psn_start=rank, psn_step=world)
    dist.barrier()
    icrc = [o.icrc_of_frame_at(buf, i * stride, flen) for i in range(n)]
    psn = [int(buf[i * stride + 37]) << 16 | int(buf[i * stride + 38]) << 8 | int(buf[i * stride + 39])
           for i in range(n)]
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.barrier()
    q.put((rank, psn, icrc, float(t[0])))
    dist.destroy_process_group()


def test_two_rank_round_robin_shards():
    world, n = 2, 50
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    # every rank saw the max of the per-rank times (max over ranks, as bench.py reports)
    assert all(r[3] == world for r in res)
    # shards are disjoint and together are the global round-robin assignment
    psns = sorted(p for r in res for p in r[1])
    assert psns == list(range(world * n))
    assert all(len(r[2]) == n and all(isinstance(c, int) for c in r[2]) for r in res)
    assert len({c for r in res for c in r[2]}) > n  # independent payload streams per rank
