"""CPU oracle for the RoCEv2 ICRC path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker / the CPU baseline.  The
product path (``roce-sim_amd/``) never imports it: the ICRC engine there is the
HIP library and it fails loudly when that library cannot run.

What it restates (reference = datenlord/roce-sim, paths relative to its root):

* ``icrc_of_frame``   -- ``BTH.compute_icrc`` (src/roce.py:192-223): the
  pseudo-packet ``Raw(FF*8) / ip.copy()`` with IP ``tos``/``ttl``/``chksum``,
  UDP ``chksum`` and BTH ``fecn``/``becn``/``resv6`` forced to all-ones
  (src/roce.py:204-211), rebuilt with a 4-byte placeholder so the IP/UDP
  lengths include the ICRC (src/roce.py:214-217), then
  ``zlib.crc32(raw(pshdr)[:-4])`` (src/roce.py:218).  A frame whose
  underlayer is not IPv4/UDP gives ICRC 0, as the reference's warning path
  does (src/roce.py:195-200, 220-223).
* ``pack_icrc``       -- ``BTH.pack_icrc`` (src/roce.py:187-190): the wire
  bytes are the CRC little-endian.
* ``build_frame``     -- the emit-side serialisation the reference gets from
  scapy: ``IP(dst)/UDP(dport=4791, sport=<QPN>)/BTH/ext/Raw``
  (src/roce_sq.py:1186-1197, src/roce_rq.py:705-731) with zero padding and
  ``padcount`` (src/roce_util.py:187-199), the BTH layout of
  src/roce.py:170-185, the extension headers of src/roce.py:236-321 and the
  ICRC trailer appended by ``BTH.post_build`` (src/roce.py:228-233).
  Scapy defaults used: IPv4 ihl 5, tos 0, id 1, flags 0, frag 0, ttl 64,
  proto 17; IP/UDP lengths and checksums computed.

Parity status (see DESIGN.md "Oracle and parity pinning"):

* The CRC arithmetic is pinned: it *is* ``zlib.crc32``, the exact function the
  reference calls (Python 3.10 stdlib, zlib 1.2.11), checked against the
  CRC-32 check value 0xCBF43926 and against an independent bitwise CRC seeded
  with 0xDEBB20E3 (``oracle/icrc_ref.c``).
* The frame bytes and the masking rule are a restatement of scapy behaviour.
  The reference cannot be imported here (scapy is not installed; an ordinary
  ``ModuleNotFoundError``, not a denial) and its own tests hold no ICRC golden
  vectors, so the serialisation/masking half is **parity unpinned** by
  reference-executed outputs.
"""

from __future__ import annotations

import struct
import zlib

ROCE_PORT = 4791  # src/roce_enum.py:14
DEFAULT_PKEY = 0xFFFF  # src/roce_enum.py:9
ICRC_SEED_REGISTER = 0xDEBB20E3  # CRC-32 register after 8 x 0xFF from init 0xFFFFFFFF

# Extension header sizes (src/roce.py:236-321)
EXT_SIZES = {
    "AETH": 4,
    "RETH": 16,
    "AtomicETH": 28,
    "AtomicAckETH": 8,
    "ImmDt": 4,
    "IETH": 4,
    "RETHImmDt": 20,
    "CNPPadding": 16,
}


def pack_icrc(icrc: int) -> bytes:
    """src/roce.py:187-190 -- struct.pack("!I", icrc)[::-1] == little-endian."""
    return struct.pack("!I", icrc & 0xFFFFFFFF)[::-1]


def masked_pseudo_packet(frame: bytes) -> bytes | None:
    """Return the bytes zlib.crc32 sees in src/roce.py:218, or None if the frame
    is not IPv4/UDP (the reference's warning path, src/roce.py:195-200, 220-223).

    ``frame`` is the wire IPv4 frame including the 4-byte ICRC slot.
    """
    b = bytearray(frame)
    if len(b) < 20 or (b[0] >> 4) != 4:
        return None
    ihl = b[0] & 0x0F
    ip_hlen = 4 * ihl
    if ihl < 5 or b[9] != 17 or len(b) < ip_hlen + 8 + 12 + 4:
        return None
    b[1] = 0xFF  # pshdr.tos = 0xFF           (src/roce.py:207)
    b[8] = 0xFF  # pshdr.ttl = 0xFF           (src/roce.py:206)
    b[10] = b[11] = 0xFF  # pshdr.chksum = 0xFFFF (src/roce.py:205)
    u = ip_hlen
    b[u + 6] = b[u + 7] = 0xFF  # pshdr[UDP].chksum = 0xFFFF (src/roce.py:208)
    bth = u + 8
    b[bth + 4] = 0xFF  # fecn=1, becn=1, resv6=0xFF&0x3F (src/roce.py:209-211)
    return b"\xff" * 8 + bytes(b[:-4])  # Raw(FF*8)/ip ... [:-4] (src/roce.py:204, 218)


def icrc_of_frame(frame: bytes) -> int:
    """BTH.compute_icrc restated (src/roce.py:192-223); returns the uint32 CRC."""
    m = masked_pseudo_packet(frame)
    if m is None:
        return 0
    return zlib.crc32(m) & 0xFFFFFFFF


_FF8_CRC = zlib.crc32(b"\xff" * 8)


def icrc_of_frame_at(buf, off: int, length: int) -> int:
    """Same rule as ``icrc_of_frame`` over ``buf[off:off+length]`` without
    copying the payload: the masked header (IP/UDP/BTH) is re-built, the rest
    is fed to zlib.crc32 as a memoryview (zlib's running-CRC argument).  This
    is the per-packet CPU baseline ("port") timed by bench.py."""
    mv = memoryview(buf)[off:off + length]
    if length < 44 or (mv[0] >> 4) != 4:
        return 0
    ihl = mv[0] & 0x0F
    hl = 4 * ihl + 8 + 12
    if ihl < 5 or mv[9] != 17 or length < hl + 4:
        return 0
    h = bytearray(mv[:hl])
    u = 4 * ihl
    h[1] = h[8] = h[10] = h[11] = 0xFF
    h[u + 6] = h[u + 7] = h[u + 12] = 0xFF
    c = zlib.crc32(h, _FF8_CRC)
    return zlib.crc32(mv[hl:length - 4], c) & 0xFFFFFFFF


def icrc_bitwise(frame: bytes) -> int:
    """Independent check: reflected CRC-32 register seeded 0xDEBB20E3 (what the
    8 x 0xFF prefix leaves), bit by bit, no tables, no zlib.  Small inputs only."""
    m = masked_pseudo_packet(frame)
    if m is None:
        return 0
    r = ICRC_SEED_REGISTER
    for byte in m[8:]:
        r ^= byte
        for _ in range(8):
            r = (r >> 1) ^ (0xEDB88320 if r & 1 else 0)
    return r ^ 0xFFFFFFFF


def verify_frame(frame: bytes) -> bool:
    """Receive-side check (new behaviour): recompute the
    ICRC over the full IPv4 frame and compare with the 4 trailing bytes."""
    if masked_pseudo_packet(frame) is None:
        return False
    return pack_icrc(icrc_of_frame(frame)) == bytes(frame[-4:])


# --------------------------------------------------------------------------
# Serialisation restatement (scapy defaults, see module docstring)
# --------------------------------------------------------------------------


def inet_checksum(data: bytes) -> int:
    if len(data) % 2:
        data += b"\0"
    s = sum(struct.unpack("!%dH" % (len(data) // 2), data))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def ip_aton(a: str) -> bytes:
    return bytes(int(x) for x in a.split("."))


def bth_bytes(
    opcode: int,
    psn: int = 0,
    dqpn: int = 0,
    solicited: int = 0,
    migreq: int = 0,
    padcount: int = 0,
    version: int = 0,
    pkey: int = DEFAULT_PKEY,
    fecn: int = 0,
    becn: int = 0,
    resv6: int = 0,
    ackreq: int = 0,
    resv7: int = 0,
) -> bytes:
    """BTH fields_desc (src/roce.py:170-184), without the FCS trailer."""
    b1 = ((solicited & 1) << 7) | ((migreq & 1) << 6) | ((padcount & 3) << 4) | (version & 0xF)
    b4 = ((fecn & 1) << 7) | ((becn & 1) << 6) | (resv6 & 0x3F)
    b8 = ((ackreq & 1) << 7) | (resv7 & 0x7F)
    return struct.pack(
        "!BBHB3sB3s",
        opcode & 0xFF,
        b1,
        pkey & 0xFFFF,
        b4,
        (dqpn & 0xFFFFFF).to_bytes(3, "big"),
        b8,
        (psn & 0xFFFFFF).to_bytes(3, "big"),
    )


def aeth_bytes(code: int = 0, value: int = 0, msn: int = 0, rsvd: int = 0) -> bytes:
    """AETH (src/roce.py:263-271): rsvd(1) code(2) value(5) msn(24)."""
    b0 = ((rsvd & 1) << 7) | ((code & 3) << 5) | (value & 0x1F)
    return bytes([b0]) + (msn & 0xFFFFFF).to_bytes(3, "big")


def reth_bytes(va: int = 0, rkey: int = 0, dlen: int = 0) -> bytes:
    return struct.pack("!QII", va, rkey, dlen)  # src/roce.py:274-280


def atomic_eth_bytes(va: int = 0, rkey: int = 0, swap: int = 0, comp: int = 0) -> bytes:
    return struct.pack("!QIQQ", va, rkey, swap, comp)  # src/roce.py:283-290


def atomic_ack_eth_bytes(orig: int = 0) -> bytes:
    return struct.pack("!Q", orig)  # src/roce.py:293-297


def immdt_bytes(data: int = 0) -> bytes:
    return struct.pack("!I", data)  # src/roce.py:300-304


def ieth_bytes(rkey: int = 0) -> bytes:
    return struct.pack("!I", rkey)  # src/roce.py:307-311


def reth_immdt_bytes(va: int = 0, rkey: int = 0, dlen: int = 0, data: int = 0) -> bytes:
    return struct.pack("!QIII", va, rkey, dlen, data)  # src/roce.py:314-321


def cnp_padding_bytes() -> bytes:
    return b"\0" * 16  # src/roce.py:236-241


def build_frame(
    src: str,
    dst: str,
    sport: int,
    bth: dict,
    ext: bytes = b"",
    payload: bytes | None = None,
    dport: int = ROCE_PORT,
    ip_id: int = 1,
    ttl: int = 64,
    tos: int = 0,
    icrc: int | None = None,
    ip_options: bytes = b"",
) -> bytes:
    """Serialise ``IP(src,dst)/UDP(sport,dport)/BTH/ext/Raw(payload)`` as scapy
    would on emit (src/roce_sq.py:1186-1197, src/roce_rq.py:705-731).

    Padding follows src/roce_util.py:187-199: only when a Raw payload is present,
    zero bytes up to a multiple of 4 and BTH.padcount = number of pad bytes.
    The ICRC trailer is computed with ``icrc_of_frame`` unless ``icrc`` is given.

    ``ip_options``: the raw bytes of scapy's ``IP(options=...)`` (the IPv4
    layer under every emit path, src/roce.py:14-31 imports it); scapy's
    ``IP.post_build`` zero-pads them to a multiple of 4 and sets
    ``ihl = header bytes / 4``.
    """
    opts = bytes(ip_options) + b"\0" * ((-len(ip_options)) % 4)
    ihl = 5 + len(opts) // 4
    bth = dict(bth)
    body = ext
    if payload is not None:
        pad = (-len(payload)) % 4
        if pad:
            bth["padcount"] = pad
        body = ext + payload + b"\0" * pad
    bth_b = bth_bytes(**bth)
    udp_len = 8 + len(bth_b) + len(body) + 4
    ip_len = 4 * ihl + udp_len
    ip_hdr = struct.pack(
        "!BBHHHBBH4s4s", 0x40 | ihl, tos, ip_len, ip_id, 0, ttl, 17, 0, ip_aton(src), ip_aton(dst)
    ) + opts
    ip_hdr = ip_hdr[:10] + struct.pack("!H", inet_checksum(ip_hdr)) + ip_hdr[12:]
    udp_wo = struct.pack("!HHHH", sport, dport, udp_len, 0)
    trailer_placeholder = b"\0\0\0\0"  # FCSField default (src/roce.py:184)
    roce = bth_b + body
    frame = ip_hdr + udp_wo + roce + trailer_placeholder
    if icrc is None:
        icrc = icrc_of_frame(frame)
    roce_with_icrc = roce + pack_icrc(icrc)
    # UDP checksum over the pseudo header (scapy in4_chksum), 0 -> 0xFFFF
    pseudo = ip_aton(src) + ip_aton(dst) + struct.pack("!BBH", 0, 17, udp_len)
    csum = inet_checksum(pseudo + udp_wo + roce_with_icrc)
    if csum == 0:
        csum = 0xFFFF
    udp = struct.pack("!HHHH", sport, dport, udp_len, csum)
    return ip_hdr + udp + roce_with_icrc


def sim_send_success_frame() -> bytes:
    """Config 1: the ``sim_send_success`` SEND_ONLY (src/case/success/sim_send_success.yaml,
    IPs from test/run.sh:9-14): 1-byte payload 0xff, ackreq=1, psn 0, dqpn 0x11,
    UDP sport = sender QPN 2."""
    return build_frame(
        src="10.1.1.48",
        dst="10.1.1.15",
        sport=2,
        bth=dict(opcode=0x04, psn=0, dqpn=0x11, ackreq=1),
        payload=b"\xff",
    )
