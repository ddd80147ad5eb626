"""GPU: more than one device, and more than one rank (BASELINE config 4 and
SURVEY.md 8(e)).

* Tests that need two or more visible devices skip cleanly on a one-GPU box:
  contexts created concurrently from one thread per device (the per-device
  kernel preparation of icrc_capi.cpp), ricrc_compute_batch_multi with
  contexts on distinct devices against the oracle on cfg4-shaped data, and
  the device-resident path on every device.
* The multi-rank path runs on any box: two ranks (gloo, one process per rank,
  each on device rank mod devices) run the ENGINE on their cfg4 shards and
  check them against the oracle, and bench.py itself is rehearsed with two
  ranks (its per-rank parity leg must report zero mismatches).
"""
import json
import os
import socket
import subprocess
import sys
import threading
from pathlib import Path

import numpy as np
import pytest

from conftest import ROOT, oracle_batch

pytestmark = pytest.mark.gpu

from roce_icrc import synth  # noqa: E402
from roce_icrc import engine as E  # noqa: E402


def _ndev() -> int:
    return E.device_count()


def _need(n: int):
    if _ndev() < n:
        pytest.skip(f"needs {n} visible GPUs ({_ndev()} here)")


def test_contexts_created_concurrently_on_every_device():
    _need(2)
    nd = _ndev()
    buf, offs, lens = synth.mixed_mtu_frames(4099, seed=31)
    want, _ = oracle_batch(buf, offs, lens)
    start = threading.Barrier(nd)
    res, errs = [None] * nd, []

    def work(d):
        try:
            start.wait()
            with E.IcrcEngine(d) as eng:
                got, st = eng.compute_batch(buf, offs, lens)
                res[d] = (got, st)
        except Exception as e:  # reported below
            errs.append((d, repr(e)))

    th = [threading.Thread(target=work, args=(d,)) for d in range(nd)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    for d in range(nd):
        got, st = res[d]
        np.testing.assert_array_equal(got, want, err_msg=f"device {d}")
        assert not st.any()


def test_compute_batch_multi_on_distinct_devices():
    """cfg4's split through the C ABI: packet i of ONE stream on device
    i mod N (ricrc_compute_batch_multi), every word against the oracle."""
    _need(2)
    nd = _ndev()
    n_total = 8192 * nd + 5
    buf, stride, flen, _ = synth.shard_frames(n_total, 0, 1)
    offs = np.arange(n_total, dtype=np.uint64) * stride
    lens = np.full(n_total, flen, np.uint32)
    want, _ = oracle_batch(buf, offs, lens)
    engines = [E.IcrcEngine(d) for d in range(nd)]
    try:
        got, st = E.compute_batch_multi(engines, buf, offs, lens)
        np.testing.assert_array_equal(got, want)
        assert not st.any()
        # a context list naming one device twice, the others once
        got2, _ = E.compute_batch_multi(engines + engines[:1], buf, offs, lens)
        np.testing.assert_array_equal(got2, want)
        # the receive-side split (ricrc_verify_batch_multi) over the stamped
        # stream, one trailer broken per device
        for i in range(n_total):
            e = int(offs[i]) + int(lens[i])
            buf[e - 4:e] = np.frombuffer(int(want[i]).to_bytes(4, "little"), np.uint8)
        bad = np.arange(nd) + 1000
        for i in bad:
            buf[int(offs[i]) + 100] ^= 1
        ok, icrc, _ = E.verify_batch_multi(engines, buf, offs, lens)
        assert ok.sum() == n_total - nd and not ok[bad].any()
        np.testing.assert_array_equal(np.delete(icrc, bad), np.delete(want, bad))
    finally:
        for e in engines:
            e.close()


def test_device_resident_on_every_device():
    _need(2)
    torch = pytest.importorskip("torch")
    n = 4096
    buf, stride, flen = synth.uniform_frames(n, 4096, seed=17)
    want, _ = oracle_batch(buf, stride=stride, length=flen, n=n)
    m_buf, m_offs, m_lens = synth.mixed_mtu_frames(3001, seed=18)
    m_want, _ = oracle_batch(m_buf, m_offs, m_lens)
    for d in range(_ndev()):
        dev = torch.device("cuda", d)
        with torch.cuda.device(dev), E.IcrcEngine(d) as eng:
            s = torch.cuda.Stream(device=dev)
            x = torch.from_numpy(buf).to(dev)
            out = torch.zeros(n, dtype=torch.int32, device=dev)
            eng.compute_strided_dev(x, stride, flen, n, out, stream=s.cuda_stream)
            mx = torch.from_numpy(m_buf).to(dev)
            mo = torch.from_numpy(m_offs.view(np.int64)).to(dev)
            ml = torch.from_numpy(m_lens.view(np.int32)).to(dev)
            mout = torch.zeros(m_offs.size, dtype=torch.int32, device=dev)
            eng.compute_batch_dev(mx, mo, ml, m_offs.size, mout, stream=s.cuda_stream)
            s.synchronize()
            np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want,
                                          err_msg=f"device {d}")
            np.testing.assert_array_equal(mout.cpu().numpy().view(np.uint32), m_want,
                                          err_msg=f"device {d}")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_worker(rank, world, port, n_total, q):
    """One rank of cfg4: its shard of the one stream, ICRCs from the ENGINE on
    device rank mod N, checked against the C oracle; results gathered over gloo."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT / "roce-sim_amd"))
    sys.path.insert(0, str(ROOT / "tests"))
    import torch.distributed as dist
    from conftest import oracle_batch as ob
    from roce_icrc import IcrcEngine
    from roce_icrc import synth as sy
    from roce_icrc import engine as eng_mod
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = rank % eng_mod.device_count()
        buf, stride, flen, gidx = sy.shard_frames(n_total, rank, world)
        with IcrcEngine(dev) as eng:
            got, st = eng.compute_strided(buf, stride, flen, gidx.size)
        want, _ = ob(buf, stride=stride, length=flen, n=gidx.size)
        mism = int((got != want).sum()) + int(st.any())
        res = [None] * world
        dist.all_gather_object(res, (rank, dev, int(gidx.size), mism, [int(x) for x in gidx[:3]]))
        dist.barrier()
        dist.destroy_process_group()
        q.put(("ok", res))
    except Exception as e:  # surfaced by the parent
        q.put(("error", f"rank {rank}: {e!r}"))


def test_two_ranks_run_the_engine_on_their_cfg4_shards():
    import torch.multiprocessing as mp
    world, n_total = 2, 2 * 20000 + 1
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, world, port, n_total, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    errs = [o[1] for o in out if o[0] != "ok"]
    assert not errs, errs
    res = sorted(out[0][1])
    assert [r[0] for r in res] == [0, 1]
    assert [r[2] for r in res] == [20001, 20000]  # packet i on rank i mod 2
    assert [r[4] for r in res] == [[0, 2, 4], [1, 3, 5]]
    assert all(r[3] == 0 for r in res), res


def test_bench_two_rank_cfg4_rehearsal(tmp_path):
    """bench.py under torch.distributed.run with two ranks (on one device when
    only one is visible): the default N > 1 workload is cfg4 and every rank's
    sampled parity leg reports zero mismatches."""
    env = dict(os.environ)
    if _ndev() < 2:
        env["ROCE_ICRC_BENCH_DEVICE"] = "0"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           str(ROOT / "bench.py"), "--gpus", "2", "--steps", "5", "--warmup", "2",
           "--packets", "40000", "--no-cpu-baseline", "--no-e2e"]
    r = subprocess.run(cmd, env=env, cwd=str(ROOT), capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["workload"].startswith("cfg4")
    assert line["config"]["packets_per_gpu"] == 40000
    assert line["parity"]["mismatches_per_rank"] == [0, 0]
    assert line["parity"]["sampled_per_rank"] == [40000, 40000]
    assert line["checks"]["pass"]


def test_plain_bench_gpus2_launches_its_own_ranks():
    """`python bench.py --gpus 2` with no launcher (the driver's form): bench.py
    starts the two ranks itself, so the line is a 2-rank cfg4 line with a
    CPU baseline over rank 0's shard (one device when only one is visible)."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    if _ndev() < 2:
        env["ROCE_ICRC_BENCH_DEVICE"] = "0"
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "5", "--warmup", "2",
           "--packets", "40000"]
    r = subprocess.run(cmd, env=env, cwd=str(ROOT), capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only, once
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["workload"].startswith("cfg4")
    assert line["parity"]["mismatches_per_rank"] == [0, 0]
    cpu = line["cpu_baseline"]
    assert cpu is not None and cpu["parity_mismatches_vs_gpu"] == 0
    assert cpu["sample"].startswith("rank 0's shard (40000 packets of 80000)")



# Ranks of the full-size rehearsal on this box: 4.  The 8-rank launch is the
# driver's (its 8-GPU scaling run); the pool's rules keep `bench.py --gpus 8`
# out of our own GPU calls, so 8 ranks are rehearsed on the CPU over gloo
# (tests/test_dist.py, the same shard split and per-rank gathers).
REHEARSAL_RANKS = 4


@pytest.mark.timeout(900)
def test_bench_multi_rank_cfg4_rehearsal_full_size(tmp_path):
    """BASELINE config 4 end to end at full per-rank size, launched as the
    driver launches it (plain `python bench.py --gpus N`, bench.py starting its
    own ranks): ONE stream of N * 2^20 4140-B packets seeded 0x1C2C0004,
    packet i on rank i mod N, 2^20 packets per rank.  With fewer than N GPUs
    every rank is pinned to device 0 (ROCE_ICRC_BENCH_DEVICE): the N-rank path
    -- rendezvous, per-rank shards, the N-way gathers, rank 0's CPU baseline
    while the others wait -- not a scaling number.  Every rank's sampled
    parity against the oracle, its device check, and the per-rank numbers of
    the line."""
    N = REHEARSAL_RANKS
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    if _ndev() < N:
        env["ROCE_ICRC_BENCH_DEVICE"] = "0"
    out_dir = ROOT / "gpurun_out"
    out_dir.mkdir(exist_ok=True)
    log = out_dir / f"rehearsal_n{N}.log"
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", str(N), "--steps", "5", "--warmup",
           "2", "--no-e2e"]
    with open(log, "w") as err:  # (the ranks' stderr: progress of a long run)
        r = subprocess.run(cmd, env=env, cwd=str(ROOT), stdout=subprocess.PIPE, stderr=err,
                           text=True, timeout=840)
    assert r.returncode == 0, log.read_text()[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    (out_dir / f"rehearsal_n{N}.json").write_text(lines[0] + "\n")
    line = json.loads(lines[0])
    assert line["n_gpus"] == N and line["config"]["workload"].startswith("cfg4")
    assert line["config"]["packets_per_gpu"] == 1 << 20
    assert line["parity"]["mismatches_per_rank"] == [0] * N
    assert line["parity"]["sampled_per_rank"] == [1 << 16] * N
    assert line["checks"]["pass"]
    cpu = line["cpu_baseline"]
    assert cpu is not None and cpu["parity_mismatches_vs_gpu"] == 0
    assert cpu["sample"].startswith(f"rank 0's shard ({1 << 20} packets of {N << 20})")
    for k in ("per_rank_GiBps", "per_rank_kernel_ms", "per_rank_kernel_GiBps", "per_rank_device"):
        assert len(line[k]) == N, k
    assert all(x > 0 for x in line["per_rank_GiBps"] + line["per_rank_kernel_ms"])
    # the aggregate: all ranks' covered bytes over the slowest rank's time
    cov = line["config"]["covered_bytes_per_gpu"]
    agg = N * cov / (line["ms_per_step"] * 1e-3) / 2**30
    assert abs(line["value"] - agg) < 0.01 * line["value"]
    assert min(line["per_rank_GiBps"]) * N <= line["value"] * 1.01


@pytest.mark.timeout(600)
def test_cfg4_stated_size_one_process():
    """BASELINE config 4 at its stated size through the HIP path without an
    8-rank launch (scripts/cfg4_one_process.py): the eight shards
    synth.shard_frames(2^23, r, 8) of the one 0x1C2C0004 stream, all resident
    on device 0 together, each through the rank's ricrc_compute_strided_dev,
    every one of the 2^23 words against the C oracle; then the same host
    stream split round robin by ricrc_compute_batch_multi over eight contexts
    on device 0, bit-exact (src/roce.py:192-219: per-packet independence)."""
    sys.path.insert(0, str(ROOT / "scripts"))
    import cfg4_one_process as c4
    res = c4.run(23, 8)
    out_dir = ROOT / "gpurun_out"
    out_dir.mkdir(exist_ok=True)
    (out_dir / "cfg4_one_process.json").write_text(json.dumps(res) + "\n")
    assert res["packets_total"] == 1 << 23 and res["packets_per_shard"] == 1 << 20
    assert res["resident"]["mismatches_per_shard"] == [0] * 8, res
    assert res["multi"]["mismatches"] == 0, res
    assert res["pass"]
