"""CPU: synthetic batches for the BASELINE configurations are well-formed
RoCEv2 frames with the layout SURVEY.md section 8(d) specifies."""
import numpy as np

import icrc_oracle as o
from roce_icrc import roce as R
from roce_icrc import synth


def test_cfg2_layout():
    buf, stride, flen = synth.uniform_frames(37, 4096, seed=synth.SEED_CFG2)
    assert stride == flen == 4140 and buf.size == 37 * 4140
    for i in (0, 1, 36):
        f = bytes(buf[i * stride:(i + 1) * stride])
        ip = R.IP(f)
        bth = ip[R.BTH]
        assert ip.len == 4140 and ip.proto == 17 and ip.ttl == 64 and ip.id == 1
        assert ip[R.UDP].dport == 4791 and ip[R.UDP].len == 4120
        assert bth.opcode == 0x01 and bth.psn == i and bth.dqpn == 0x11 and bth.pkey == 0xFFFF
        assert len(bth[R.Raw].load) == 4096
        assert o.masked_pseudo_packet(f) is not None
    assert synth.covered_bytes(np.full(37, 4140)) == 37 * 4136


def test_round_robin_shard_psns():
    world = 4
    seen = []
    for rank in range(world):
        buf, stride, _ = synth.uniform_frames(5, 64, seed=1 + rank, psn_start=rank, psn_step=world)
        seen += [R.IP(bytes(buf[i * stride:(i + 1) * stride]))[R.BTH].psn for i in range(5)]
    assert sorted(seen) == list(range(world * 5))


def test_cfg4_shards_are_the_one_global_stream():
    """cfg4: ONE stream seeded 0x1C2C0004, packet i -> rank i mod N (SURVEY
    8(d)); every rank's shard is exactly its rows of that stream."""
    n_total, world = 37, 4
    whole, stride, flen = synth.uniform_frames(n_total, 4096, seed=synth.SEED_CFG4)
    rows = whole.reshape(n_total, flen)
    got = {}
    for rank in range(world):
        buf, s, fl, idx = synth.shard_frames(n_total, rank, world, chunk=4)
        assert s == fl == flen and list(idx) == list(range(rank, n_total, world))
        sh = buf.reshape(-1, flen)
        assert (sh == rows[idx]).all(), rank
        for k, i in enumerate(idx):
            got[int(i)] = R.IP(bytes(sh[k]))[R.BTH].psn
    assert got == {i: i for i in range(n_total)}
    one, _, _, idx = synth.shard_frames(n_total, 0, 1)
    assert (one == whole).all() and idx.size == n_total


def test_cfg3_mixed_mtu():
    n = 4000
    buf, offs, lens = synth.mixed_mtu_frames(n, seed=synth.SEED_CFG3)
    pay = lens.astype(int) - 44
    assert set(np.unique(pay)) == set(synth.MTUS)
    assert (offs[1:] == offs[:-1] + lens[:-1]).all()  # packed back to back
    mean_c = synth.covered_bytes(lens) / n
    assert abs(mean_c - 1627.2) < 60  # E[C] = 1627.2 B
    for i in (0, 1, 2, n - 1):
        f = bytes(buf[int(offs[i]):int(offs[i] + lens[i])])
        ip = R.IP(f)
        assert ip.len == lens[i] and ip[R.BTH].opcode == 0x07 and ip[R.BTH].psn == i
        assert f[-4:] == b"\0\0\0\0"


def test_cfg5_small():
    buf, stride, flen = synth.uniform_frames(10, 64, seed=synth.SEED_CFG5)
    assert flen == 108
    assert R.IP(bytes(buf[:108]))[R.BTH].opcode == 0x01
