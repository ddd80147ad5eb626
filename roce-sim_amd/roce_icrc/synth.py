"""Synthetic RoCEv2 frame batches for the BASELINE.json configurations.

Frames follow the emit-side layout of datenlord/roce-sim:
``IP(dst)/UDP(dport=4791, sport=<QPN>)/BTH/payload`` (src/roce_sq.py:1186-1197)
with scapy's IPv4 defaults (ihl 5, tos 0, id 1, flags 0, ttl 64, proto 17) and
the BTH layout of src/roce.py:170-185.  Full-MTU payloads need no padding
(src/roce_util.py:187-199).  The UDP checksum is left 0 ("no checksum" in
IPv4): it is one of the ICRC-masked fields (src/roce.py:208), so its value
cannot change an ICRC.  The ICRC trailer is left zero unless a caller fills it.

Configurations:
  cfg2 / cfg4  RC SEND_MIDDLE (0x01), 4096-B random payload, stride 4140
  cfg3         RDMA_WRITE_MIDDLE (0x07), MTU drawn from {256..4096}, packed
  cfg5         SEND_MIDDLE-shaped, 64-B payload, stride 108
"""

from __future__ import annotations

import struct

import numpy as np

ROCE_PORT = 4791
IP_HDR = 20
UDP_HDR = 8
BTH_HDR = 12
HDR = IP_HDR + UDP_HDR + BTH_HDR  # 40
ICRC = 4

SEED_CFG2 = 0x1C2C0001
SEED_CFG3 = 0x1C2C0003
SEED_CFG4 = 0x1C2C0004
SEED_CFG5 = 0x1C2C0005
MTUS = (256, 512, 1024, 2048, 4096)


def _ip_checksum(hdr: bytes) -> int:
    s = sum(struct.unpack("!10H", hdr))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def header_template(payload_len: int, opcode: int, src="10.1.1.48", dst="10.1.1.15",
                    sport: int = 2, dqpn: int = 0x11, pkey: int = 0xFFFF) -> np.ndarray:
    """40-byte IPv4 + UDP + BTH header of a frame carrying `payload_len` bytes
    (already a multiple of 4).  PSN is 0; callers write it per packet."""
    frame_len = HDR + payload_len + ICRC
    ip = struct.pack("!BBHHHBBH4s4s", 0x45, 0, frame_len, 1, 0, 64, 17, 0,
                     bytes(int(x) for x in src.split(".")), bytes(int(x) for x in dst.split(".")))
    ip = ip[:10] + struct.pack("!H", _ip_checksum(ip)) + ip[12:]
    udp = struct.pack("!HHHH", sport, ROCE_PORT, frame_len - IP_HDR, 0)
    bth = struct.pack("!BBHB3sB3s", opcode, 0, pkey, 0, dqpn.to_bytes(3, "big"), 0, b"\0\0\0")
    return np.frombuffer(ip + udp + bth, dtype=np.uint8).copy()


def _random_bytes(rng: np.random.Generator, nbytes: int) -> np.ndarray:
    words = rng.integers(0, 2**63 - 1, size=(nbytes + 7) // 8, dtype=np.int64, endpoint=True)
    return words.view(np.uint8)[:nbytes]


def _write_psn(hdr_rows: np.ndarray, psn: np.ndarray) -> None:
    psn = psn.astype(np.uint32) & 0xFFFFFF
    hdr_rows[:, 37] = (psn >> 16).astype(np.uint8)
    hdr_rows[:, 38] = (psn >> 8).astype(np.uint8)
    hdr_rows[:, 39] = psn.astype(np.uint8)


def uniform_frames(n: int, payload_len: int = 4096, opcode: int = 0x01, seed: int = SEED_CFG2,
                   psn_start: int = 0, psn_step: int = 1,
                   chunk: int = 1 << 16) -> tuple[np.ndarray, int, int]:
    """n back-to-back frames of identical length (cfg2/cfg4/cfg5).

    Returns (buffer, stride, frame_len) with stride == frame_len.  PSN of
    packet i is (psn_start + i * psn_step) mod 2^24 (psn_step = N for the
    round-robin shard of rank psn_start out of N GPUs)."""
    assert payload_len % 4 == 0
    frame_len = HDR + payload_len + ICRC
    buf = np.empty(n * frame_len, dtype=np.uint8)
    rows = buf.reshape(n, frame_len)
    tmpl = header_template(payload_len, opcode)
    rng = np.random.Generator(np.random.PCG64(seed))
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        r = rows[s:e]
        r[:, :HDR] = tmpl
        _write_psn(r, psn_start + psn_step * np.arange(s, e, dtype=np.int64))
        r[:, HDR:HDR + payload_len] = _random_bytes(rng, (e - s) * payload_len).reshape(
            e - s, payload_len)
        r[:, HDR + payload_len:] = 0
    return buf, frame_len, frame_len


def shard_frames(n_total: int, rank: int, world: int, payload_len: int = 4096,
                 opcode: int = 0x01, seed: int = SEED_CFG4,
                 chunk: int = 1 << 14,
                 out: np.ndarray | None = None) -> tuple[np.ndarray, int, int, np.ndarray]:
    """cfg4: ONE global stream of n_total frames built
    like cfg2 from `seed`, packet i going to rank i mod world; returns this
    rank's shard (packets rank, rank + world, ... in order) as (buffer,
    stride, frame_len, global packet indices).

    The global stream is the one ``uniform_frames(n_total, payload_len,
    seed=seed)`` builds (payload words of packet i = 64-bit outputs
    [i W, (i + 1) W) of PCG64(seed), W = payload_len / 8, each shifted right
    by one bit as ``Generator.integers(0, 2**63 - 1)`` returns them; PSN = i
    mod 2^24), so a rank generates only its own packets: the generator jumps
    over the other ranks' words with ``PCG64.advance``.  At world = 1 the
    shard is the whole uniform_frames batch, byte for byte.  ``out``: a
    uint8 buffer of the shard's size to build it in (e.g. a region of one
    shared block holding every shard)."""
    assert payload_len % 8 == 0 and 0 <= rank < world
    idx = np.arange(rank, n_total, world, dtype=np.int64)
    n = idx.size
    frame_len = HDR + payload_len + ICRC
    if out is None:
        buf = np.empty(n * frame_len, dtype=np.uint8)
    else:
        buf = out.reshape(-1)
        if buf.dtype != np.uint8 or buf.size != n * frame_len:
            raise ValueError(f"out must be {n * frame_len} uint8 bytes")
    rows = buf.reshape(n, frame_len)
    tmpl = header_template(payload_len, opcode)
    W = payload_len // 8
    bg = np.random.PCG64(seed)
    if n:
        bg.advance(int(idx[0]) * W)
    skip = (world - 1) * W
    words = np.empty((min(chunk, max(n, 1)), W), dtype=np.uint64)
    one = np.uint64(1)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        for k in range(e - s):
            words[k] = bg.random_raw(W)
            if skip:
                bg.advance(skip)
        r = rows[s:e]
        r[:, :HDR] = tmpl
        _write_psn(r, idx[s:e])
        r[:, HDR:HDR + payload_len] = (words[:e - s] >> one).view(np.uint8)
        r[:, HDR + payload_len:] = 0
    return buf, frame_len, frame_len, idx


def mixed_mtu_frames(n: int, mtus=MTUS, opcode: int = 0x07, seed: int = SEED_CFG3,
                     chunk: int = 1 << 16) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """cfg3: n frames, payload = MTU drawn uniformly from `mtus`, packed
    back-to-back.  Returns (buffer, offsets u64, lens u32)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    mt = np.asarray(mtus, dtype=np.int64)
    sel_mtu = rng.integers(0, len(mtus), size=n)
    pay = mt[sel_mtu]
    lens = (HDR + pay + ICRC).astype(np.uint32)
    offsets = np.zeros(n, dtype=np.uint64)
    if n > 1:
        np.cumsum(lens[:-1], out=offsets[1:])
    total = int(offsets[-1] + lens[-1]) if n else 0
    buf = _random_bytes(rng, total).copy()  # payload bytes everywhere, headers below
    tmpls = np.stack([header_template(int(m), opcode) for m in mtus])
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        base = offsets[s:e].astype(np.int64)
        rows = tmpls[sel_mtu[s:e]].copy()
        _write_psn(rows, np.arange(s, e, dtype=np.int64))
        buf[base[:, None] + np.arange(HDR)[None, :]] = rows
        tail = base + lens[s:e].astype(np.int64) - ICRC
        buf[tail[:, None] + np.arange(ICRC)[None, :]] = 0
    return buf, offsets, lens


def covered_bytes(lens) -> int:
    """Sum of C_i = IPv4 total length - 4."""
    return int(np.asarray(lens, dtype=np.int64).sum() - ICRC * np.asarray(lens).size)
