"""CPU: the reference-mirror packet API (roce_icrc.roce) -- serialisation and
dissection against the oracle's independent restatement.  ICRC values here are
explicit (no GPU); the GPU tests cover compute_icrc through the engine."""
import struct

import pytest

import icrc_oracle as o
from roce_icrc import roce as R


def _ref(bth_kw, ext=b"", payload=None, sport=2):
    return o.build_frame("10.1.1.48", "10.1.1.15", sport, bth_kw, ext=ext, payload=payload)


def _mirror(pkt, sport=2, icrc=None):
    l3 = R.l3_packet(pkt, dst="10.1.1.15", sport=sport, src="10.1.1.48")
    l3[R.BTH].__dict__["icrc"] = icrc
    return bytes(l3)


@pytest.mark.parametrize("payload", [b"", b"\xff", b"ab", b"abc", b"abcd", bytes(range(255))])
def test_send_only_bytes_match_oracle(payload):
    ref = _ref(dict(opcode=0x04, psn=0, dqpn=0x11, ackreq=1), payload=payload or None)
    icrc = struct.unpack("<I", ref[-4:])[0]
    pkt = R.BTH(opcode=R.opcode("RC", "SEND_ONLY")[0], psn=0, dqpn=0x11, ackreq=1)
    if payload:
        pkt = pkt / R.Raw(load=payload)
    assert _mirror(pkt, icrc=struct.unpack("!I", ref[-4:])[0]) == ref
    assert icrc == o.icrc_of_frame(ref)


def test_every_ext_header_layout():
    cases = [
        (R.AETH(code="NAK", value=2, msn=9), o.aeth_bytes(3, 2, 9), 0x11),
        (R.RETH(va=0x1122334455667788, rkey=0xAABBCCDD, dlen=4096),
         o.reth_bytes(0x1122334455667788, 0xAABBCCDD, 4096), 0x0C),
        (R.AtomicETH(va=5, rkey=6, swap=7, comp=8), o.atomic_eth_bytes(5, 6, 7, 8), 0x13),
        (R.ImmDt(data=0xDEADBEEF), o.immdt_bytes(0xDEADBEEF), 0x05),
        (R.IETH(rkey=0x42), o.ieth_bytes(0x42), 0x17),
        (R.RETHImmDt(va=1, rkey=2, dlen=3, data=4), o.reth_immdt_bytes(1, 2, 3, 4), 0x0B),
        (R.CNPPadding(), o.cnp_padding_bytes(), 0x81),
    ]
    for hdr, ref_bytes, op in cases:
        assert bytes(hdr) == ref_bytes
        ref = _ref(dict(opcode=op, psn=7, dqpn=3), ext=ref_bytes)
        pkt = R.BTH(opcode=op, psn=7, dqpn=3) / hdr
        assert _mirror(pkt, icrc=struct.unpack("!I", ref[-4:])[0]) == ref


def test_atomic_ack_stack_and_padding():
    ref = _ref(dict(opcode=0x12, psn=1, dqpn=2),
               ext=o.aeth_bytes(0, 31, 3) + o.atomic_ack_eth_bytes(77))
    pkt = R.BTH(opcode=0x12, psn=1, dqpn=2) / R.AETH(code="ACK", value=31, msn=3) / R.AtomicAckETH(orig=77)
    assert _mirror(pkt, icrc=struct.unpack("!I", ref[-4:])[0]) == ref
    p = R.add_padding_if_needed(R.BTH(opcode=0x04) / R.Raw(load=b"\x01\x02\x03\x04\x05"))
    assert p[R.BTH].padcount == 3 and p[R.Raw].load == b"\x01\x02\x03\x04\x05\0\0\0"


def test_dissect_roundtrip_and_bindings():
    ref = _ref(dict(opcode=0x0D, psn=0x123456, dqpn=0xABCDEF, solicited=1),
               ext=o.aeth_bytes(0, 31, 5), payload=b"xyz")
    ip = R.IP(ref)
    bth = ip[R.BTH]
    assert ip.src == "10.1.1.48" and ip[R.UDP].dport == 4791
    assert (bth.opcode, bth.psn, bth.dqpn, bth.padcount, bth.solicited) == (0x0D, 0x123456, 0xABCDEF, 1, 1)
    assert isinstance(bth.payload, R.AETH) and bth[R.AETH].msn == 5
    assert bth[R.Raw].load == b"xyz\0"
    # FCSField: BTH.icrc is the trailer read big-endian (the byte-swapped CRC)
    assert bth.icrc == struct.unpack("!I", ref[-4:])[0]
    assert R.BTH.pack_icrc(o.icrc_of_frame(ref)) == ref[-4:]
    for op, cls in [(0x0A, R.RETH), (0x0B, R.RETHImmDt), (0x13, R.AtomicETH), (0x81, R.CNPPadding),
                    (0x09, R.ImmDt), (0x16, R.IETH), (0x01, R.Raw)]:
        assert R._BTH_BINDINGS.get(op, R.Raw) is cls


@pytest.mark.parametrize("opts", [
    b"\x01\x01\x01\x00",                      # NOP NOP NOP EOL (ihl 6)
    [R.IPOption(b"\x94\x04\x00\x00")],        # router alert (ihl 6)
    [R.IPOption(b"\x07\x07\x04"), R.IPOption(b"\x0a\x0b\x0c\x0d")],  # record route, zero pad
    b"\x01" * 40,                              # the largest header (ihl 15)
])
def test_ipv4_options_build_and_dissect(opts):
    """IP(options=...) under the RoCE stack (scapy's IP layer, src/roce.py:14-31;
    the emit wrap src/roce_sq.py:1189-1193): ihl > 5, options zero-padded to
    whole dwords, lengths and checksums over the longer header -- byte for
    byte the oracle's restatement -- and dissect keeps the option bytes."""
    raw = opts if isinstance(opts, bytes) else b"".join(bytes(x) for x in opts)
    payload = bytes(range(37))
    ref = o.build_frame("10.1.1.48", "10.1.1.15", 9, dict(opcode=0x0A, psn=5, dqpn=0x77),
                        ext=o.reth_bytes(0x1000, 0x22, 37), payload=payload, ip_options=raw)
    ihl = 5 + (len(raw) + 3) // 4
    assert ref[0] == 0x40 | ihl and len(ref) == 4 * ihl + 8 + 12 + 16 + 40 + 4
    pkt = R.add_padding_if_needed(
        R.BTH(opcode=0x0A, psn=5, dqpn=0x77) / R.RETH(va=0x1000, rkey=0x22, dlen=37) / R.Raw(load=payload))
    l3 = R.IP(src="10.1.1.48", dst="10.1.1.15", options=opts) / R.UDP(dport=4791, sport=9) / pkt
    l3[R.BTH].__dict__["icrc"] = struct.unpack("!I", ref[-4:])[0]
    assert bytes(l3) == ref
    assert struct.unpack("<I", ref[-4:])[0] == o.icrc_of_frame(ref) == o.icrc_bitwise(ref)
    d = R.IP(ref)
    assert d.ihl == ihl and b"".join(bytes(x) for x in d.options) == ref[20:4 * ihl]
    assert d[R.UDP].dport == 4791 and d[R.BTH].psn == 5 and d[R.RETH].dlen == 37
    assert d[R.Raw].load == payload + b"\0\0\0"
    assert bytes(d) == ref  # round trip: the dissected packet rebuilds the same frame
    # the wire frame compute_icrc hands the engine is the frame with a zero slot
    assert R.wire_frame(l3, l3[R.UDP], bytes(l3[R.BTH])[:-4] + b"\0" * 4)[:4 * ihl] == \
        ref[:10] + bytes(2) + ref[12:4 * ihl]


def test_opcode_table_and_cnp():
    assert R.opcode("RC", "SEND_ONLY") == (0x04, "RC_SEND_ONLY")
    assert R.opcode("XRC", "FETCH_ADD")[0] == 0xB4
    assert R._bth_opcodes[0x81] == "CNP" and len(R._bth_opcodes) == 83  # src/roce.py:79-165
    c = R.cnp(0x77)
    assert c.opcode == 0x81 and c.becn == 1 and c.dqpn == 0x77 and isinstance(c.payload, R.CNPPadding)


def test_warning_path_without_ip_underlayer():
    # BTH directly over UDP with no IP, or bare: warning + zero ICRC, no engine needed
    with pytest.warns(UserWarning):
        out = bytes(R.BTH(opcode=0x11) / R.AETH())
    assert out[-4:] == b"\0\0\0\0"
    with pytest.warns(UserWarning):
        out = bytes(R.UDP(dport=4791) / R.BTH(opcode=0x11) / R.AETH())
    assert out[-4:] == b"\0\0\0\0"
