"""CPU, gloo: the multi-GPU path of bench.py -- BASELINE config 4 (SURVEY.md
8(d)/(e)): ONE stream seeded 0x1C2C0004, packet i on rank i mod N
(synth.shard_frames, each rank generating only its own packets), no data-path
collective, a barrier, a MAX-reduce of the timing and bench.py's own per-rank
gathers (gather_ranks / rank_fields) -- with the CPU oracle as each rank's
worker.  World sizes 2 and 8: the 8-rank launch itself is the driver's 8-GPU
run; this is its rehearsal without a card."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root))
    sys.path.insert(0, str(root / "roce-sim_amd"))
    sys.path.insert(0, str(root / "oracle"))
    try:
        import torch
        import bench
        import icrc_oracle as o
        from roce_icrc import synth
        dist.init_process_group("gloo", rank=rank, world_size=world)
        buf, stride, flen, gidx = synth.shard_frames(n_total, rank, world, payload_len=256)
        dist.barrier()
        icrc = [o.icrc_of_frame_at(buf, i * stride, flen) for i in range(gidx.size)]
        psn = [int(buf[i * stride + 37]) << 16 | int(buf[i * stride + 38]) << 8
               | int(buf[i * stride + 39]) for i in range(gidx.size)]
        t_local = 0.001 * (rank + 1)
        t = torch.tensor([t_local], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        covered = gidx.size * (flen - 4)
        ranks = bench.gather_ranks(dist, world, rank, rank, t_local, [t_local / 5] * 5, covered)
        fields = bench.rank_fields(ranks, 5)
        dist.barrier()
        q.put((rank, [int(x) for x in gidx], psn, icrc, float(t[0]), fields, buf.tobytes()))
        dist.destroy_process_group()
    except Exception as e:  # surfaced by the parent
        q.put((rank, "error", repr(e)))


@pytest.mark.parametrize("world", [2, 8])
def test_round_robin_shards_of_one_stream(world):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root / "oracle"))
    import icrc_oracle as o
    from roce_icrc import synth
    n_total = 50 * world + 3  # ragged: the first 3 ranks hold one packet more
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    errs = [r for r in res if r[1] == "error"]
    assert not errs, errs
    res.sort(key=lambda r: r[0])
    # every rank saw the max of the per-rank times (max over ranks, as bench.py reports)
    assert all(r[4] == 0.001 * world for r in res)
    # packet i on rank i mod N, each shard in stream order, together the stream
    for rank, gidx, psn, *_ in res:
        assert gidx == list(range(rank, n_total, world))
        assert psn == gidx
    # byte for byte the frames of the one stream (uniform_frames, cfg4 seed),
    # so the shards' ICRCs are the stream's ICRCs
    whole, stride, flen = synth.uniform_frames(n_total, 256, seed=synth.SEED_CFG4)
    want = [o.icrc_of_frame_at(whole, i * stride, flen) for i in range(n_total)]
    got = [None] * n_total
    for rank, gidx, _, icrc, _, _, raw in res:
        rows = np.frombuffer(raw, np.uint8).reshape(len(gidx), flen)
        np.testing.assert_array_equal(rows, whole.reshape(n_total, flen)[gidx])
        for g, c in zip(gidx, icrc):
            got[g] = c
    assert got == want
    # bench.py's per-rank keys, identical on every rank, in rank order
    fields = [r[5] for r in res]
    assert all(f == fields[0] for f in fields)
    f = fields[0]
    assert f["per_rank_device"] == list(range(world))
    assert len(f["per_rank_GiBps"]) == len(f["per_rank_kernel_ms"]) == world
    cov = [len(r[1]) * (flen - 4) for r in res]
    for k in range(world):
        assert f["per_rank_GiBps"] == pytest.approx(
            [round(c * 5 / (0.001 * (i + 1)) / 2**30, 3) for i, c in enumerate(cov)])
        assert f["per_rank_kernel_ms"][k] == pytest.approx(0.2 * (k + 1), abs=1e-4)
